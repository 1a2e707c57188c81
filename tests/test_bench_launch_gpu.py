"""bench.py's multi-GPU contract on the builder's one GPU: ``--gpus 2`` with no
outer launcher starts two ranks itself (torch.distributed.run child process),
every rank runs the DDP train step, rank 0 prints ONE JSON line with n_gpus = 2
and the max-over-ranks time. RCCL refuses two ranks on one device, so this
rehearsal uses ``--backend gloo``; on an 8-GPU node the same path runs RCCL."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _run(extra):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo", "--steps", "2",
           "--warmup", "1", "--batch", "4", "--points", "256", "--emb", "64", "--no-roofline-leg",
           "--no-fp32-leg", *extra]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(300)
def test_bench_self_launch_two_ranks_weak():
    r = _run([])
    assert r["n_gpus"] == 2 and r["scaling"] == "weak"
    assert r["config"]["global_batch"] == 8 and r["config"]["batch_per_gpu"] == 4
    assert r["value"] > 0 and r["config"]["parallelism"] == "dp2"
    # fwd+bwd graph per rank + one all-reduce of the flat gradient buffer
    assert r["launch"] == "hip_graph+allreduce" and r["replicas_in_sync"] is True


@pytest.mark.timeout(300)
def test_bench_self_launch_two_ranks_ddp():
    r = _run(["--no-graph"])
    assert r["n_gpus"] == 2 and r["launch"] == "eager" and r["replicas_in_sync"] is True


@pytest.mark.timeout(300)
def test_bench_self_launch_two_ranks_strong_syncbn():
    r = _run(["--scaling", "strong", "--sync-bn"])
    assert r["n_gpus"] == 2 and r["scaling"] == "strong"
    assert r["config"]["global_batch"] == 4 and r["config"]["batch_per_gpu"] == 2
    assert r["config"]["parallelism"] == "dp2+syncbn"
    assert r["launch"] == "eager" and r["replicas_in_sync"] is True
