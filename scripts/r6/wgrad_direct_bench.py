"""Split-free wgrad (ops.conv_wgrad_direct) vs the production split-K wgrad + reduce, per layer.

For each batch size: the 192 -> 192 3x3 layer and the 5x5 first layer (48 real planes of 64), timed with
HIP events over 200 back-to-back launches (layer inputs rotate over 8 buffers so the operands do not sit
in L2 between calls).  Prints one JSON line per (B, layer, plan)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from alphago_amd import ops  # noqa: E402


def timed(fn, n=200):
    for _ in range(10):
        fn(0)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(n):
        fn(i)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3  # us


def main():
    ops.load()
    dev = torch.device("cuda")
    S = 19
    bs = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,2,4,8,16").split(",")]
    for B in bs:
        for name, Cin, cin_real, Cout, K, Pin in (("3x3_192", 192, 192, 192, 3, 1), ("5x5_first", 64, 48, 192, 5, 2)):
            xs = [ops.to_padded(torch.randn(B, cin_real, S, S, device=dev).bfloat16().float(), Pin, Cin)
                  for _ in range(8)]
            dzs = [ops.to_padded(torch.randn(B, Cout, S, S, device=dev).bfloat16().float(), 1) for _ in range(8)]
            gw = torch.zeros(Cout, cin_real, K, K, device=dev)
            gb = torch.zeros(Cout, device=dev)
            M = B * S * S
            var, ns = ops.wgrad_config(M, Cout, Cin, K, cin_real if cin_real < Cin else 0)
            slab = torch.empty(ns, K * K, Cout, Cin, device=dev)
            dbs = torch.empty(ns, Cout, device=dev)

            def splitk(i):
                ops.conv_wgrad(xs[i % 8], dzs[i % 8], slab, dbs, K, S, Pin, 1,
                               cin_real=cin_real if cin_real < Cin else 0, variant=var)
                ops.conv_wgrad_reduce(slab, dbs, gw, gb, 1.0, 0.0)

            def splitk_only(i):
                ops.conv_wgrad(xs[i % 8], dzs[i % 8], slab, dbs, K, S, Pin, 1,
                               cin_real=cin_real if cin_real < Cin else 0, variant=var)

            rows = {"splitk+reduce": timed(splitk), "splitk_only": timed(splitk_only)}
            ref = gw.clone()
            for ks in (1, 2, 4):
                rows["direct_k%d" % ks] = timed(lambda i: ops.conv_wgrad_direct(xs[i % 8], dzs[i % 8], gw, gb, K, S,
                                                                               Pin, 1, ksub=ks))
            # same result as the split plan (last inputs: buffer (n-1) % 8 for both)
            splitk(199)
            ref = gw.clone()
            ops.conv_wgrad_direct(xs[199 % 8], dzs[199 % 8], gw, gb, K, S, Pin, 1, ksub=1)
            err = ((gw - ref).abs().max() / ref.abs().max()).item()
            print(json.dumps({"B": B, "layer": name, "variant": var, "nsplit": ns,
                              "us": {k: round(v, 2) for k, v in rows.items()}, "rel_err_vs_splitk": err}), flush=True)


if __name__ == "__main__":
    main()
