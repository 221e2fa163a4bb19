#!/usr/bin/env python3
"""Per-call cost of the OpenMP CPU backend (BASELINE config #1: the 1024^2
fp32 transpose, blocked, preallocated output) under different OpenMP thread
policies, each in a fresh process so the runtime reads its environment at
load time. Prints one JSON line per setting: median / min / max of single
calls after warm-up, with and without torch imported first.

    python benchmarks/omp_floor.py [--calls 60] [--threads 1 2 4 8 16]

Why: with libgomp's default wait policy (spin ~300k iterations before
sleeping) single calls in this container's VM took ~64 ms (16 x 4-ms
scheduler ticks) whenever the host was busy, against 0.25 ms otherwise --
in a torch process or not (VERDICT r5 "What's missing" #1)."""
import argparse
import json
import os
import subprocess
import sys

CHILD = r"""
import ctypes, json, os, sys, time
import numpy as np
if os.environ.get("PROBE_TORCH") == "1":
    import torch  # noqa: F401 -- its libgomp loads first, as in a framework process
lib = ctypes.CDLL(sys.argv[1])
f = lib.cme_cpu_transpose_f32
f.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int] * 3
n = 1024
x = np.arange(n * n, dtype=np.float32)
y = np.empty_like(x)
for _ in range(5):
    f(x.ctypes.data, y.ctypes.data, n, n, 1)
assert np.array_equal(y.reshape(n, n), x.reshape(n, n).T)
ts = []
for _ in range(int(sys.argv[2])):
    t0 = time.perf_counter()
    f(x.ctypes.data, y.ctypes.data, n, n, 1)
    ts.append((time.perf_counter() - t0) * 1e3)
ts.sort()
print(json.dumps({"median_ms": round(ts[len(ts) // 2], 4), "min_ms": round(ts[0], 4), "max_ms": round(ts[-1], 4)}))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=60)
    ap.add_argument("--threads", type=int, nargs="+", default=[1, 2, 4, 8, 16])
    ap.add_argument("--lib", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "2012-04_stanford_cme213_amd", "lib", "libcme213_cpu.so"))
    args = ap.parse_args()
    base = {k: v for k, v in os.environ.items() if not k.startswith(("OMP_", "GOMP_"))}
    settings = [("default", {}), ("passive", {"OMP_WAIT_POLICY": "PASSIVE"}),
                ("spin10k", {"GOMP_SPINCOUNT": "10000"})]
    print(json.dumps({"cpus_affinity": len(os.sched_getaffinity(0)), "nproc": os.cpu_count(),
                      "env_OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}), flush=True)
    for torch_first in ("0", "1"):
        for th in args.threads:
            for name, env in settings:
                e = dict(base, OMP_NUM_THREADS=str(th), PROBE_TORCH=torch_first, **env)
                r = subprocess.run([sys.executable, "-c", CHILD, args.lib, str(args.calls)], env=e,
                                   capture_output=True, text=True, timeout=300)
                rec = {"policy": name, "threads": th, "torch_first": torch_first == "1"}
                if r.returncode == 0:
                    rec.update(json.loads(r.stdout.strip().splitlines()[-1]))
                else:
                    rec["error"] = r.stderr[-300:]
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
