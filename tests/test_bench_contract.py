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
    if mode == "halo":  # 64x64 grid in 3 row blocks: neighbours only, about one grid row each way
        assert rec["max_peers_per_rank"] == 2 and rec["max_halo_values_per_rank"] <= 2 * 64 + 2


def _launch_gpu(nproc, extra):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", str(nproc), "--steps", "20", "--warmup", "3", "--spinup", "0", "--grid", "2048", *extra]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("nproc,extra", [(2, []), (4, ["--method", "2", "--tblock", "4"])])
def test_bench_multirank_shared_gpu_ipc(gpu, nproc, extra):
    """The driver's N>1 bench flow (torch.distributed.run, one process per
    rank, native loop after its bitwise self-test) rehearsed on ONE GPU: every
    rank on cuda:0, gloo control plane, IPC halo transport."""
    rec = _launch_gpu(nproc, ["--share-gpu", *extra])
    assert rec["n_gpus"] == nproc and rec["sanity_ok"] is True
    assert rec["native_selftest"] is True and rec["selftest"] is True
    assert rec["config"]["loop"] == "native-ipc" and rec["config"]["rehearsal_shared_gpu"] is True
    assert rec["config"]["transport"] == "ipc" and rec["config"]["schedule"].split()[0] in ("fused", "events")


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_single_gpu_selftest(gpu):
    """N = 1 (the driver's BENCH run): the timed path -- one native
    multi-pass call per loop -- passes its bitwise self-test against single
    FMA steps and names its schedule."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "9", "--warmup", "5", "--grid", "2048",
           "--spinup", "0.05"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    assert rec["selftest"] is True and rec["sanity_ok"] is True
    assert rec["steps"] == 9 and rec["warmup"] == 5
    assert rec["config"]["schedule"] and rec["config"]["transport"] == "none"
