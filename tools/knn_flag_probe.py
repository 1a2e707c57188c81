"""Count the rows knn_kernel flags for the exact fix-up (rank-0 id = -1 before
knn_fix_kernel) on the bench's layer inputs. Needs a probe build of libdgx
without the fix-up launch (DGX_LIB=...): python tools/knn_flag_probe.py"""
import os
import sys
import types

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
import torch  # noqa: E402

from dgx import synth  # noqa: E402
from dgx.ops import knn_raw  # noqa: E402
from dgx.edgeconv import debug_capture, set_debug_capture, edgeconv_stack  # noqa: E402
from models.dgcnn import DGCNN  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
x = torch.from_numpy(synth.cube_clouds(32, 1024, 0)).to(dev).permute(0, 2, 1).contiguous()
for k in (20, 16, 40):
    idx = knn_raw(x, k, out_dtype=torch.int32)
    print("xyz k", k, "flagged rows", int((idx[..., 0] == -1).sum()))
g = torch.Generator(device="cpu").manual_seed(1)
for C in (64, 128):
    f = torch.randn(32, C, 1024, generator=g).to(dev)
    idx = knn_raw(f, 20, out_dtype=torch.int32)
    print("gauss C", C, "flagged rows", int((idx[..., 0] == -1).sum()))
m = DGCNN(types.SimpleNamespace(emb_dim=1024, k=20)).to(dev).train()
d = {}
set_debug_capture(d)
with torch.no_grad():
    y = m(x)
set_debug_capture(None)
for key in sorted(k for k in d if isinstance(k, tuple)):
    idx = d[key][0]
    print("dgcnn block", key, "flagged rows", int((idx.view(-1, 20)[:, 0] == -1).sum()))
