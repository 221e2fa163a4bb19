#!/usr/bin/env python3
"""AddressSanitizer + UndefinedBehaviorSanitizer run of the native CPU
backend -- the host-side equivalent of the ``cuda-memcheck`` the course
teaches (``slides/Lecture06.pdf`` slides 2-3; SURVEY §5 "race detection /
sanitizers"). GPU code is not instrumented (device sanitizers are not
available on this pool).

1. builds ``csrc/cpu/*.cpp`` with g++ ``-O1 -g -fsanitize=address,undefined
   -fno-sanitize-recover=all`` into ``build/asan/libcme213_cpu.so``;
2. runs the CPU test suite (``-m "not gpu"``) with that library
   (``CME_CPU_LIB``), the sanitizer runtimes preloaded into the (uninstrumented)
   Python interpreter, and every report fatal.

    python scripts/asan_cpu.py [pytest args...]      # or: make test-asan
"""
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
OUT = REPO / "build" / "asan"
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]


def runtime(name: str) -> str:
    p = subprocess.run(["g++", f"-print-file-name={name}"], capture_output=True, text=True, check=True).stdout.strip()
    if not os.path.isabs(p):
        raise SystemExit(f"sanitizer runtime {name} not found")
    return p


def build() -> Path:
    OUT.mkdir(parents=True, exist_ok=True)
    objs = []
    for src in sorted((REPO / "csrc" / "cpu").glob("*.cpp")):
        obj = OUT / (src.stem + ".o")
        cmd = ["g++", "-O1", "-g", "-std=c++17", "-fPIC", "-fopenmp", "-ffp-contract=off", *SAN,
               f"-I{REPO / 'csrc' / 'include'}", "-c", str(src), "-o", str(obj)]
        subprocess.run(cmd, check=True)
        objs.append(str(obj))
    lib = OUT / "libcme213_cpu.so"
    subprocess.run(["g++", "-shared", "-fPIC", "-fopenmp", *SAN, "-o", str(lib), *objs], check=True)
    return lib


def main() -> int:
    lib = build()
    env = dict(os.environ)
    env.update(
        CME_CPU_LIB=str(lib),
        CME_AUTOBUILD="0",
        LD_PRELOAD=":".join([runtime("libasan.so"), runtime("libubsan.so")]),
        # python itself is not instrumented: its allocations look like leaks
        ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0",
        UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
        OMP_NUM_THREADS=env.get("OMP_NUM_THREADS", "4"),
    )
    args = sys.argv[1:] or ["tests", "-x", "-q", "-m", "not gpu", "-p", "no:cacheprovider"]
    return subprocess.call([sys.executable, "-m", "pytest", *args], cwd=REPO, env=env)


if __name__ == "__main__":
    sys.exit(main())
