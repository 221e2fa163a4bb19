#!/usr/bin/env python3
"""ISA check: is every LDS write waited for (s_waitcnt lgkmcnt(0)) before
the next s_barrier on every control-flow path?

hipcc's __syncthreads() puts `s_waitcnt lgkmcnt(0)` before `s_barrier`, but
drops it when the barrier heads a loop and the LDS write is at the end of
the loop body (profiles/lds_broadcast_isa_r6.md): then a wave can pass the
barrier while another wave's ds_write is still in flight. This walks the
gfx950 assembly of each kernel (basic blocks, fall-through and branch edges)
from every LDS write (ds_write*, ds_* atomics) and reports the s_barrier
reached without an lgkmcnt(0) wait.

    python scripts/check_lds_barriers.py csrc/hip/sort.hip [more.hip ...]   # compiles with hipcc -S
    python scripts/check_lds_barriers.py --asm file.s                        # an existing listing

Prints one JSON line per kernel: barriers, LDS writes, and the unwaited
(write line, barrier line) pairs. Exit 1 if any kernel has one.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

_LDS_WRITE = re.compile(r"^ds_(write|store|add|sub|rsub|inc|dec|min|max|and|or|xor|mskor|wrxchg|cmpst|cmpswap|"
                        r"pk_add|add_rtn|condxchg)")
_LABEL = re.compile(r"^(\.LBB\d+_\d+):")
_FUNC = re.compile(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$")


def parse_functions(asm: str) -> dict[str, list[tuple[int, str]]]:
    """kernel name -> [(source line number, instruction or '.LBB label:')]"""
    funcs: dict[str, list[tuple[int, str]]] = {}
    cur = None
    for no, raw in enumerate(asm.splitlines(), 1):
        line = raw.split(";")[0].rstrip()
        m = _FUNC.match(line)
        if m and not line.startswith("."):
            cur = m.group(1)
            funcs[cur] = []
            continue
        if cur is None:
            continue
        s = line.strip()
        if not s:
            continue
        if _LABEL.match(s):
            funcs[cur].append((no, s))
        elif s.startswith(".Lfunc_end"):
            cur = None
        elif not s.startswith("."):
            funcs[cur].append((no, s))
    return funcs


def unwaited(body: list[tuple[int, str]]) -> tuple[int, int, list[tuple[int, int]]]:
    """(#barriers, #LDS writes, [(write line, barrier line)] reached with no
    lgkmcnt(0) in between on some path)."""
    labels = {s[:-1]: i for i, (_, s) in enumerate(body) if _LABEL.match(s)}

    def succ(i):
        """indices control can go to after instruction i"""
        s = body[i][1]
        op = s.split()[0]
        if op == "s_endpgm" or op.startswith("s_setpc"):
            return []
        if op == "s_branch":
            return [labels[s.split()[1]] for _ in [0] if s.split()[1] in labels]
        out = []
        if op.startswith("s_cbranch") and len(s.split()) > 1 and s.split()[1] in labels:
            out.append(labels[s.split()[1]])
        if i + 1 < len(body):
            out.append(i + 1)
        return out

    bad = []
    nbar = sum(1 for _, s in body if s == "s_barrier")
    writes = [i for i, (_, s) in enumerate(body) if _LDS_WRITE.match(s)]
    for w in writes:
        seen = set()
        stack = succ(w)
        while stack:
            i = stack.pop()
            if i in seen:
                continue
            seen.add(i)
            s = body[i][1]
            if s.startswith("s_waitcnt") and "lgkmcnt(0)" in s:
                continue
            if s == "s_barrier":
                bad.append((body[w][0], body[i][0]))
                continue
            stack.extend(succ(i))
    return nbar, len(writes), bad


def check_asm(asm: str, src: str) -> list[dict]:
    out = []
    for name, body in parse_functions(asm).items():
        nbar, nw, bad = unwaited(body)
        if nbar == 0:
            continue
        out.append({"source": src, "kernel": name, "barriers": nbar, "lds_writes": nw,
                    "unwaited": sorted(set(bad))})
    return out


def compile_asm(src: str) -> str:
    with tempfile.TemporaryDirectory() as d:
        s = os.path.join(d, "k.s")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics",
                        f"-I{os.path.join(REPO, 'csrc', 'include')}", "--cuda-device-only", "-S", src, "-o", s],
                       check=True, capture_output=True)
        with open(s) as f:
            return f.read()


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("sources", nargs="*")
    ap.add_argument("--asm", nargs="*", default=[])
    args = ap.parse_args()
    recs = []
    for a in args.asm:
        with open(a) as f:
            recs += check_asm(f.read(), a)
    for s in args.sources:
        recs += check_asm(compile_asm(s), os.path.relpath(s, REPO))
    rc = 0
    for r in recs:
        print(json.dumps(r))
        rc |= bool(r["unwaited"])
    return int(rc)


if __name__ == "__main__":
    sys.exit(main())
