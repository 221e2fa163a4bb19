#!/usr/bin/env python3
"""Sweep the streamN chunk rule for strong-scaled subdomains: runs
``bench_dist_rank.py`` (one rank's compute schedule, exchange off) in a fresh
process per setting of CME_STREAMN_ROUNDS / CME_STREAMN_MINCHUNK /
CME_STREAMN_CHUNK (read once per process by the native library) and prints
one JSON line per (setting, world).

    python benchmarks/tune_dist_rank.py [--out gpurun_out/tune_dist_rank.jsonl]
"""
import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

SETTINGS = [
    {},  # default rule
    {"CME_STREAMN_MINCHUNK": "32"},  # the round-1 rule (3 rounds, >= 32-row chunks)
    {"CME_STREAMN_MINCHUNK": "96"},
    {"CME_STREAMN_MINCHUNK": "128"},
    {"CME_STREAMN_ROUNDS": "2"},
    {"CME_STREAMN_ROUNDS": "1"},
    {"CME_STREAMN_ROUNDS": "4", "CME_STREAMN_MINCHUNK": "48"},
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--methods", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--steps", type=int, default=150)
    ap.add_argument("--settings", default=None, help="JSON list of env dicts (default: the built-in sweep)")
    ap.add_argument("--world", default="1 2 4 8")
    ap.add_argument("--extra", default="", help="extra bench_dist_rank.py arguments")
    args = ap.parse_args()
    settings = json.loads(args.settings) if args.settings else SETTINGS
    out = open(args.out, "a") if args.out else None
    for method in args.methods:
        for st in settings:
            env = dict(os.environ)
            env.update(st)
            cmd = [sys.executable, os.path.join(HERE, "bench_dist_rank.py"), "--method", str(method), "--steps",
                   str(args.steps), "--world", *args.world.split(), *args.extra.split()]
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(p.stderr[-2000:], file=sys.stderr)
                raise SystemExit(p.returncode)
            for line in p.stdout.splitlines():
                if line.startswith("{"):
                    rec = json.loads(line)
                    rec["setting"] = st
                    s = json.dumps(rec)
                    print(s, flush=True)
                    if out:
                        out.write(s + "\n")
                        out.flush()


if __name__ == "__main__":
    main()
