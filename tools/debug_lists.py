import ctypes, os, sys
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DGX_LIB"] = os.path.join(REPO, "tools", "libdgx_dbg.so")
sys.path[:0] = [REPO, os.path.join(REPO, "dgcnn.pytorch_amd")]
from dgx import _native, synth  # noqa
from dgx.ops import knn_raw  # noqa
L = _native.lib()
L.dgx_knn_set_debug.argtypes = [ctypes.c_void_p]
pts = synth.tie_clouds(32, 1024, 1)
for (b, row) in ((9, 787), (14, 225)):
    x = torch.from_numpy(pts[b:b + 1]).permute(0, 2, 1).cuda()
    dbg = torch.zeros(1024 * 4 * 20 * 2, device="cuda")
    L.dgx_knn_set_debug(ctypes.c_void_p(dbg.data_ptr()))
    idx = knn_raw(x, 20).cpu().numpy()[0]
    torch.cuda.synchronize()
    d = dbg.cpu().numpy().reshape(1024, 4, 2, 20)
    print("row", row, "final", idx[row].tolist())
    for g in range(4):
        print("  g", g, "ids", d[row, g, 1].astype(int).tolist())
        print("     vals", d[row, g, 0].tolist()[:6])
