"""One conv shape on tile 40 (weight-stationary) and the automatic tile, N launches each (PMC target)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from alphago_amd import ops  # noqa: E402

ops.load()
dev = torch.device("cuda")
B, C, S, K = int(sys.argv[1]), int(sys.argv[2]), 19, 3
w = torch.randn(C, C, K, K, device=dev) * 0.05
wf = ops.packed_weight_like(w, C, C)
ops.pack_weights([w.contiguous()], [wf])
wws = ops.ws_packed_like(wf)
ops.ws_pack([wf], [wws])
b = torch.randn(C, device=dev) * 0.1
x = ops.padded_empty(B, S, 1, C, dev).normal_()
y = ops.padded_empty(B, S, 1, C, dev)
mb = torch.zeros(B * (S + 2) ** 2 * ops.mbits_words(C), dtype=torch.int32, device=dev)
for tile in (40, 0):
    for _ in range(20):
        ops.conv_fwd(x, wws if tile == 40 else wf, b, y, K, S, 1, 1, mbits=mb, tile=tile)
torch.cuda.synchronize()
