"""Phase timing of the push-form scatter (edge_bwd_push_kernel) against the
pull form at cfg2 layer shapes: DGX_PUSH_SKIP bits drop phases (1 exponent
pass, 2 push, 4 in-edge loop, 8 Q staging, 16 atomics only); results are wrong
with any bit set — timing only."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "dgcnn.pytorch_amd"))
import test_scatter_push_gpu as T  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    cuda = torch.device("cuda:0")
    for Co in (64, 256):
        for packed in (True,):
            S = T._setup(cuda, 32, 1024, 20, Co, packed=packed)
            pull = timeit(lambda: T._pull(S, packed))
            res = {}
            for skip in (0, 1, 2, 16, 4, 8, 2 | 4, 1 | 2 | 4, 1 | 2 | 4 | 8):
                os.environ["DGX_PUSH_SKIP"] = str(skip)
                res[skip] = timeit(lambda: T._push(S, packed))
            os.environ.pop("DGX_PUSH_SKIP")
            print(f"Co {Co} packed {packed}: pull {pull:.1f} us; push by skip mask: "
                  + ", ".join(f"{k}:{v:.1f}" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
