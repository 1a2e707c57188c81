"""RCCL on the one GPU of the builder's box (reference
main_partseg_dist.py:189-196, 486): a world-size-1 "nccl" process group runs
the engine's multi-GPU code paths on hardware (tests/_rccl_worker.py), and
bench.py's --rccl-world1 takes its N>1 branch.

* flat (bench.py's hip_graph+allreduce step) and ddp (torch DDP buckets) are
  BIT-EQUAL to the plain single-process step after 3 SGD steps: output,
  gradients, parameters, running statistics. At world 1 the all-reduce is the
  identity and the 1/world scale multiplies by 1.0, so any difference would be
  a defect of the distributed path itself (buffer aliasing, a missed or
  doubled gradient, a stale capture).
* sync / syncg: SyncBatchNorm forced to synchronise at world 1. The fp64 sums
  all-reduced from the C++ op give bit-identical results eagerly and with the
  collectives captured inside the HIP graph; against the plain step they
  differ only by the fp64-vs-fp32 statistics finalize (a rounding of the BN
  scale), held to 1e-4 — the N>1 SyncBatchNorm tolerance of
  tests/test_ddp_gpu.py.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import REPO, rel_err

pytestmark = pytest.mark.gpu


def _worker(tmp_path, precision):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "_rccl_worker.py"), str(tmp_path), precision],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    return torch.load(os.path.join(tmp_path, "rccl1.pt"), weights_only=True)


def _bitwise(a, b, what):
    assert torch.equal(a["y"], b["y"]), f"{what}: output"
    for sect in ("grads", "params", "buffers"):
        for n, t in a[sect].items():
            assert torch.equal(t, b[sect][n]), f"{what}: {sect} {n}"


@pytest.mark.timeout(300)
@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_rccl_world1_paths_bit_equal(tmp_path, precision):
    res = _worker(tmp_path, precision)
    plain = res["plain"]
    _bitwise(res["flat"], plain, "flat-buffer graph + RCCL all-reduce")
    _bitwise(res["ddp"], plain, "DDP over RCCL")
    _bitwise(res["syncg"], res["sync"], "SyncBatchNorm collectives in graph vs eager")
    errs = {"y": rel_err(res["sync"]["y"], plain["y"])}
    for n, t in plain["grads"].items():
        errs[n] = rel_err(res["sync"]["grads"][n], t)
    for n, t in plain["buffers"].items():
        if t.is_floating_point():
            errs[n] = rel_err(res["sync"]["buffers"][n], t)
    print(json.dumps({k: float(v) for k, v in errs.items()}))
    assert max(errs.values()) < 1e-4, errs


@pytest.mark.timeout(300)
@pytest.mark.parametrize("sync", [False, True])
def test_bench_rccl_world1(sync):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--rccl-world1", "--steps", "3", "--warmup", "2",
           "--batch", "8", "--no-roofline-leg", "--no-fp32-leg", "--no-edgeconv-leg", "--no-posemb-leg",
           "--no-attention-leg", "--no-eager-baseline", "--no-cpu-baseline"] + (["--sync-bn"] if sync else [])
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    r = json.loads(lines[0])
    assert r["n_gpus"] == 1 and r["config"]["backend"] == "rccl" and r["value"] > 0
    assert r["launch"] == "hip_graph+allreduce" + ("(+syncbn collectives in graph)" if sync else "")
    assert r["replicas_in_sync"] is True
    assert r["config"]["parallelism"] == "dp1" + ("+syncbn" if sync else "")
