"""Host simulation of the kNN kernel's selection schedule (no GPU): counts the
insertion rounds a wave pays (max FIFO depth over its 64 lanes per flush) for
the two-half / 8-list design, so list length, FIFO depth and flush trigger can
be tuned offline. python tools/knn_select_sim.py [C] [k] [KL] [QCAP] [trigger]"""
import sys

import numpy as np

sys.path[:0] = ["dgcnn.pytorch_amd"]
from dgx import synth  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 64
k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
KL = int(sys.argv[3]) if len(sys.argv) > 3 else 12
QCAP = int(sys.argv[4]) if len(sys.argv) > 4 else 16
TRIG = int(sys.argv[5]) if len(sys.argv) > 5 else QCAP - 4
FORCE = {int(v) for v in sys.argv[6].split(",")} if len(sys.argv) > 6 and sys.argv[6] else set()
MMODE = sys.argv[7] if len(sys.argv) > 7 else "min"
N = 1024
if C == 3:
    x = synth.cube_clouds(1, N, 0)[0].astype(np.float64)           # (N, 3)
else:
    x = synth.relu_normal(3, (1, C, N))[0].T.astype(np.float64)    # (N, C)
pd = 2 * x @ x.T - (x * x).sum(1)[None, :] - (x * x).sum(1)[:, None]
m = -(-k // 8)
tot_rounds, tot_flush, tot_adm = 0, 0, 0
for q0 in range(0, 64, 16):                      # 4 query groups
    qs = np.arange(q0, q0 + 16)
    ntile = N // 16
    lists = {h: np.full((16, 4, KL), -np.inf) for h in (0, 1)}
    fifo = {h: [[[] for _ in range(4)] for _ in range(16)] for h in (0, 1)}
    thr = {h: np.full((16, 4), -np.inf) for h in (0, 1)}
    pub = {h: np.full(16, -np.inf) for h in (0, 1)}
    rounds = {0: 0, 1: 0}
    for step in range(ntile // 2):
        for h in (0, 1):
            s = h + 2 * step
            for g in range(4):
                for r in range(4):
                    j = s * 16 + g + 4 * r
                    v = pd[qs, j]
                    for qi in range(16):
                        if v[qi] >= thr[h][qi, g]:
                            fifo[h][qi][g].append(v[qi])
            cnt = np.array([[len(fifo[h][qi][g]) for g in range(4)] for qi in range(16)])
            last = step == ntile // 2 - 1
            if cnt.max() > TRIG or last or step in FORCE:
                rounds[h] += cnt.max()
                tot_flush += 1
                tot_adm += cnt.sum()
                for qi in range(16):
                    for g in range(4):
                        L = np.sort(np.concatenate([lists[h][qi, g], fifo[h][qi][g]]))[::-1][:KL]
                        lists[h][qi, g] = L
                        fifo[h][qi][g] = []
                if MMODE == "min":
                    tm = lists[h][:, :, m - 1].min(1)
                    pub[h] = tm
                    t = np.minimum(tm, pub[1 - h])
                elif MMODE == "max2":  # max(own 4 lists' min m4-th, all 8 lists' min m-th)
                    m4 = -(-k // 4)
                    own = lists[h][:, :, m4 - 1].min(1)
                    tm = lists[h][:, :, m - 1].min(1)
                    pub[h] = tm
                    t = np.maximum(own, np.minimum(tm, pub[1 - h]))
                elif MMODE == "union":  # exact k-th of all 8 lists (partner's as of its last flush)
                    allv = np.sort(np.concatenate([lists[0].reshape(16, -1), lists[1].reshape(16, -1)], 1), axis=1)[:, ::-1]
                    t = allv[:, k - 1]
                else:  # exact k-th over the wave's 4 lists + partner bound
                    allv = np.sort(lists[h].reshape(16, -1), axis=1)[:, ::-1]
                    pub[h] = allv[:, k // 2 - 1]   # >= k/2 elements in this wave's lists
                    t = np.minimum(pub[h], pub[1 - h])
                thr[h] = np.maximum(t[:, None], lists[h][:, :, KL - 1])
    tot_rounds += rounds[0] + rounds[1]
waves = 8
print(f"C={C} k={k} KL={KL} QCAP={QCAP} trig>{TRIG}: rounds/wave {tot_rounds / waves:.1f}, "
      f"flushes/wave {tot_flush / waves:.1f}, admitted/lane {tot_adm / waves / 64:.1f}, "
      f"insert VALU/wave ~{tot_rounds / waves * (5 * KL + 8):.0f}")
