"""Host profile of the eager SL training step at a small batch: cProfile over N steps of the bench
trainer (random data), top functions by total time."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from alphago_amd.models.nets import PolicyNet  # noqa: E402
from alphago_amd.train.engine import make_policy_trainer  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
dev = torch.device("cuda")
torch.manual_seed(0)
net = PolicyNet(48, board=19, filters_per_layer=192, layers=12)
tr = make_policy_trainer(net, B, 0.003, 0.0, backend="hip", device=dev)
planes = torch.randint(0, 2, (B, 48, 19, 19), dtype=torch.uint8, device=dev)
tgt = torch.randint(0, 361, (B,), device=dev, dtype=torch.int32)
for _ in range(30):
    tr.step(planes, tgt)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(200):
    tr.step(planes, tgt)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
