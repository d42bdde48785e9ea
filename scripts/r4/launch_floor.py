"""Where the small-batch forward's time goes: per-kernel cost of a HIP-graph chain of trivial kernels,
the split-K forward at B = 1 over split counts, and tiles 64 / 42 at large inference batches.
One JSON line per measurement.  Usage: python scripts/r4/launch_floor.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from alphago_amd import ops  # noqa: E402


def graph_us(run, reps=20):
    run()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def main():
    ops.load()
    dev = torch.device("cuda")
    t = torch.zeros(1, device=dev)
    for n in (12, 48):
        us = graph_us(lambda: [t.add_(1) for _ in range(n)])
        print(json.dumps({"what": "trivial_kernel_chain", "kernels": n, "us_per_kernel": round(us / n, 2)}), flush=True)
    S, F, L = 19, 192, 12
    w = torch.randn(F, F, 3, 3, device=dev) * 0.05
    wf = ops.packed_weight_like(w, F, F)
    ops.pack_weights([w], [wf])
    bias = torch.zeros(F, device=dev)
    for B in (1, 2, 4):
        M = B * S * S
        xs = [ops.padded_empty(B, S, 1, F, dev) for _ in range(2)]
        xs[0][:, 1:S + 1, 1:S + 1].normal_()
        for ns in (1, 2, 3, 6, 9, 18, 27):
            ws = torch.empty(ns * M * F, device=dev)

            def run():
                for l in range(L):
                    ops.conv_fwd_splitk(xs[l % 2], wf, bias, xs[(l + 1) % 2], 3, S, 1, 1, ops.MODE_BIAS_RELU, None,
                                        ws, ns)
            print(json.dumps({"what": "splitk", "B": B, "nsplit": ns, "us_per_layer": round(graph_us(run) / L, 2)}),
                  flush=True)
    for B in (512, 1024, 2048):
        xs = [ops.padded_empty(B, S, 1, F, dev) for _ in range(2)]
        xs[0][:, 1:S + 1, 1:S + 1].normal_()
        for tile in (0, 64, 42):
            def run():
                for l in range(L):
                    ops.conv_fwd(xs[l % 2], wf, bias, xs[(l + 1) % 2], 3, S, 1, 1, tile=tile)
            print(json.dumps({"what": "tile", "B": B, "tile": tile, "us_per_layer": round(graph_us(run, 10) / L, 2)}),
                  flush=True)


if __name__ == "__main__":
    main()
