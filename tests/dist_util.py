"""Helpers to run a function on N gloo ranks (CPU, 127.0.0.1) in subprocesses."""
import os
import socket
import sys
import traceback

import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def init_single_rank(backend: str = "nccl") -> None:
    """World-1 process group on cuda:0 (no-op if one exists). A port that
    free_port() saw free can be taken again before the store binds it
    (EADDRINUSE); the rendezvous then fails before any GPU work, so another
    port is tried."""
    import torch
    import torch.distributed as dist

    if dist.is_initialized():
        return
    for attempt in range(5):
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1",
                          LOCAL_RANK="0")
        try:
            dist.init_process_group(backend, rank=0, world_size=1, device_id=torch.device("cuda", 0))
            return
        except dist.DistNetworkError:
            if attempt == 4:
                raise


def _worker(rank, world, port, fn, args, q):
    try:
        if REPO not in sys.path:
            sys.path.insert(0, REPO)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank), OMP_NUM_THREADS="2")
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)  # gloo default; GPU tests add nccl groups
        out = fn(rank, world, *args)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok", out))
    except Exception:  # pragma: no cover - surfaced in the parent
        q.put((rank, "err", traceback.format_exc()))


def run_ranks(fn, world: int = 2, args=(), timeout: float = 300):
    """Run fn(rank, world, *args) on `world` spawned gloo ranks; returns the
    per-rank results. A rendezvous port taken between free_port() and the
    store's bind (EADDRINUSE: a host-side race, nothing ran) is retried with
    a fresh port, twice at most."""
    for attempt in range(3):
        try:
            return _run_ranks_once(fn, world, args, timeout)
        except RuntimeError as e:
            if "EADDRINUSE" not in str(e) or attempt == 2:
                raise


def _run_ranks_once(fn, world, args, timeout):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, status, out = q.get(timeout=timeout)
            if status != "ok":
                raise RuntimeError(f"rank {rank} failed:\n{out}")
            results[rank] = out
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [results[r] for r in range(world)]
