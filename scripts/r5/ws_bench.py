"""Per-layer GPU time of the weight-stationary conv (tile 40) vs the automatic tiles at small batches:
a chain of 11 192 -> 192 3x3 forwards (and bitmask dgrads), 11 distinct weight tensors as in the net,
captured in one HIP graph, replayed."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from alphago_amd import ops  # noqa: E402

ops.load()
dev = torch.device("cuda")
S = 19
for C, K, Cin in [(c, 3, c) for c in (int(v) for v in os.environ.get("WS_WIDTHS", "192,160").split(","))]:
    for B in [int(v) for v in os.environ.get("WS_BATCHES", "1,4,8,16,32,64").split(",")]:
        ws = [(torch.randn(C, Cin, K, K, device=dev) * 0.05).contiguous() for _ in range(11)]
        wfs = [ops.packed_weight_like(w, Cin, C) for w in ws]
        wds = [ops.packed_weight_like(w, Cin, C, True) for w in ws]
        ops.pack_weights(ws, wfs, wds)
        wfs_ws = [ops.ws_packed_like(w) for w in wfs]
        wds_ws = [ops.ws_packed_like(w) for w in wds]
        ops.ws_pack(wfs + wds, wfs_ws + wds_ws)
        b = torch.randn(C, device=dev) * 0.1
        xs = [ops.padded_empty(B, S, 1, C, dev) for _ in range(2)]
        xs[0].normal_()
        mb = torch.zeros(B * (S + 2) ** 2 * ops.mbits_words(C), dtype=torch.int32, device=dev)
        res = {"C": C, "B": B}
        for tile in [int(v) for v in os.environ.get("WS_TILES", "0,40").split(",")]:
            for mode in (("fwd",) if tile > 1000 else ("fwd", "dgrad")):
                def chain():
                    for i in range(11):
                        if tile > 1000:  # kernel-lab probes of tile 40 (forward only)
                            ops.lab().conv_fwd(xs[i % 2], wfs_ws[i], b, None, xs[(i + 1) % 2], K, S, 1, 1, 0, mb,
                                               tile)
                        elif mode == "fwd":
                            ops.conv_fwd(xs[i % 2], wfs_ws[i] if tile == 40 else wfs[i], b, xs[(i + 1) % 2], K, S, 1,
                                         1, mbits=mb, tile=tile)
                        else:
                            ops.conv_fwd(xs[i % 2], wds_ws[i] if tile == 40 else wds[i], None, xs[(i + 1) % 2], K, S,
                                         1, 1, mode=ops.MODE_MASKBITS, mbits=mb, tile=tile)
                chain()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    chain()
                for _ in range(3):
                    g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    g.replay()
                e1.record()
                e1.synchronize()
                res["%s_t%d_us" % (mode, tile)] = round(e0.elapsed_time(e1) / 20 / 11 * 1e3, 2)
        print(json.dumps(res), flush=True)
