"""bench.py contract: the multi-rank control flow (torch.distributed.run
launch, decomposition, barriers, max-over-ranks timing, one JSON line from
rank 0) exercised end to end on CPU ranks (gloo + OpenMP backend)."""
import json
import os
import subprocess
import sys

import pytest

from dist_util import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(nproc, extra):
    env = dict(os.environ, OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", str(nproc), "--steps", "5", "--warmup", "1", "--grid", "192", "--device", "cpu", *extra]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # exactly one JSON line (rank 0)
    return json.loads(lines[0])


@pytest.mark.parametrize("nproc,extra", [(2, []), (4, ["--method", "2"]), (3, ["--mode", "sync", "--tblock", "1"])])
def test_bench_multirank_cpu(nproc, extra):
    rec = _launch(nproc, extra)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in rec
    assert rec["n_gpus"] == nproc and rec["steps"] == 5 and rec["warmup"] == 1
    assert rec["sanity_ok"] is True and rec["value"] > 0
    assert rec["config"]["loop"] == "torch.distributed"


@pytest.mark.parametrize("mode", ["halo", "allgather"])
def test_dist_spmv_bench_cpu(mode):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, "benchmarks", "bench_dist_spmv.py"),
           "--grid", "64", "--steps", "3", "--warmup", "1", "--device", "cpu", "--mode", mode]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["n_gpus"] == 3 and rec["max_abs_err"] < 1e-4
