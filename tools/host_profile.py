"""Host-side (CPU) cost of one eager cfg2 train step: torch.profiler CPU time
per Python op / function, to see where the eager step's launch overhead goes.
python tools/host_profile.py [steps]"""
import os
import sys
import time
import types

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
from dgx import precision, synth  # noqa: E402
from models.dgcnn import DGCNN  # noqa: E402

dev = torch.device("cuda:0")
precision.set("bf16")
torch.manual_seed(0)
m = DGCNN(types.SimpleNamespace(emb_dim=1024, k=20)).to(dev).train()
opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, fused=True)
x = torch.from_numpy(synth.cube_clouds(32, 1024, 0)).to(dev).permute(0, 2, 1)
gy = torch.rand(32, 1024, 1024, device=dev) - 0.5


def step():
    opt.zero_grad(set_to_none=True)
    m(x).backward(gy)
    opt.step()


for _ in range(5):
    step()
torch.cuda.synchronize()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
# host time per step with the GPU kept far ahead: time the issue loop only
t0 = time.perf_counter()
for _ in range(n):
    step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"issue {1e3 * (t1 - t0) / n:.3f} ms/step (host), wall {1e3 * (t2 - t0) / n:.3f} ms/step", flush=True)
import cProfile  # noqa: E402
import pstats  # noqa: E402
pr = cProfile.Profile()
pr.enable()
for _ in range(10):
    step()
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(45)
