"""Per-layer GPU time of the 192 -> 192 3x3 forward at small batches on each small tile, measured as
HIP-graph replays of 12 back-to-back convs (no host dispatch in the timing, unlike the eager
small_batch_kbench.py); TILES=a,b,... picks the tiles (0 = the automatic choice; default 64, 36 =
32 pixels, 38 = 36 + split-K; the narrow-N tiles 39 / 42 measured here were removed, profiles/r4/README.md).  One JSON line per (B, tile).  Usage: python scripts/r4/small_tile_graph_bench.py [B ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from alphago_amd import ops  # noqa: E402


def main():
    ops.load()
    dev = torch.device("cuda")
    S, F, L = 19, int(os.environ.get("WIDTH", "192")), 12  # WIDTH=160: the value net's padded width
    bs = [int(b) for b in sys.argv[1:]] or [1, 4, 16, 64]
    w = torch.randn(F, F, 3, 3, device=dev) * 0.05
    wf = ops.packed_weight_like(w, F, F)
    ops.pack_weights([w], [wf])
    bias = torch.zeros(F, device=dev)
    for B in bs:
        M = B * S * S
        xs = [ops.padded_empty(B, S, 1, F, dev) for _ in range(2)]
        xs[0][:, 1:S + 1, 1:S + 1].normal_()
        for tile in [int(t) for t in os.environ.get("TILES", "64,36,38").split(",")]:
            ns = 0
            if tile == 38:
                tiles = (M + 31) // 32 * (F // ops.conv_n_tile(F))
                ns = max(1, min(9, -(-512 // tiles)))
                ws = torch.empty(ns * M * F, device=dev)

            def run():
                for l in range(L):
                    x, y = xs[l % 2], xs[(l + 1) % 2]
                    if tile == 38:
                        ops.conv_fwd_splitk(x, wf, bias, y, 3, S, 1, 1, ops.MODE_BIAS_RELU, None, ws, ns)
                    else:
                        ops.conv_fwd(x, wf, bias, y, 3, S, 1, 1, tile=tile)
            run()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                run()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1000.0 / 20 / L
            print(json.dumps({"B": B, "tile": tile, "nsplit": ns, "us_per_layer": round(us, 2)}), flush=True)


if __name__ == "__main__":
    main()
