"""Small-batch conv kernels (round 4): per-layer time of the 192 -> 192 3x3 forward / bitmask dgrad
on each small-M tiling (64 = 2-buffer 64-pixel tile, 65 / 130 = the 64 / 128-pixel tiles on a 4 / 3-slot
LDS ring, 128) and of the wgrad + split-K reduce (variant 0 with the min-stages splits vs the ring
variant 9 with ops.wgrad_config's longer splits).  One JSON line per (B, kernel, config).
Usage: python scripts/r4/small_batch_kbench.py [B ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from alphago_amd import ops  # noqa: E402


def timeit(fn, iters=200, warm=20):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


def main():
    ops.load()
    dev = torch.device("cuda")
    S, F = 19, 192
    bs = [int(b) for b in sys.argv[1:]] or [1, 4, 16, 64, 256]
    w = torch.randn(F, F, 3, 3, device=dev) * 0.05
    wf, wd = ops.packed_weight_like(w, F, F), ops.packed_weight_like(w, F, F, True)
    ops.pack_weights([w], [wf], [wd])
    bias = torch.zeros(F, device=dev)
    for B in bs:
        M = B * S * S
        x = ops.padded_empty(B, S, 1, F, dev)
        x[:, 1:S + 1, 1:S + 1].normal_()
        y = ops.padded_empty(B, S, 1, F, dev)
        mb = torch.zeros(B * (S + 2) ** 2 * ops.mbits_words(F), dtype=torch.int32, device=dev)
        for tile in (64, 65, 130, 128):
            t_f = timeit(lambda: ops.conv_fwd(x, wf, bias, y, 3, S, 1, 1, mbits=mb, tile=tile))
            t_d = timeit(lambda: ops.conv_fwd(x, wd, None, y, 3, S, 1, 1, mode=ops.MODE_MASKBITS, mbits=mb,
                                              tile=tile))
            print(json.dumps({"B": B, "kernel": "fwd", "tile": tile, "us": round(t_f, 2)}), flush=True)
            print(json.dumps({"B": B, "kernel": "dgrad", "tile": tile, "us": round(t_d, 2)}), flush=True)
        gw = torch.zeros(F, F, 3, 3, device=dev)
        gb = torch.zeros(F, device=dev)
        cfgs = [(0, ops.wgrad_nsplit(M, F, F, 3))] + [(9, max(1, (M + 31) // 32 // st)) for st in (8, 16, 32)]
        for var, ns in cfgs:
            slab = torch.empty(ns, 9, F, F, device=dev)
            dbs = torch.zeros(ns, F, device=dev)
            t_w = timeit(lambda: ops.conv_wgrad(x, y, slab, dbs, 3, S, 1, 1, variant=var))
            t_r = timeit(lambda: ops.conv_wgrad_reduce(slab, dbs, gw, gb, 1.0, 0.0))
            print(json.dumps({"B": B, "kernel": "wgrad", "variant": var, "nsplit": ns, "us": round(t_w, 2),
                              "reduce_us": round(t_r, 2)}), flush=True)


if __name__ == "__main__":
    main()
