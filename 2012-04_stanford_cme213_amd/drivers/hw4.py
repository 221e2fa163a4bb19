"""hw4 sort drivers (argv and output lines of the reference programs).

    python -m cme213x radixsort [n [numBits]] [--gpu]
    python -m cme213x mergesort sortThreshold mergeThreshold n doSerial [--gpu]
"""
from __future__ import annotations

import sys
import time

import numpy as np
import torch


def radixsort_main(argv=None) -> int:
    from ..ops.sort import sort

    argv = list(sys.argv[1:] if argv is None else argv)
    gpu = "--gpu" in argv
    argv = [x for x in argv if x != "--gpu"]
    n = int(argv[0]) if len(argv) >= 1 else 40_000_000
    bits = int(argv[1]) if len(argv) >= 2 else 8
    print(f"n_elements: {n}\nnumBits: {bits}")
    keys = torch.from_numpy(np.random.default_rng(0).integers(0, 2**31 - 1, n, dtype=np.int64).astype(np.int32))
    t0 = time.perf_counter()
    ref = np.sort(keys.numpy())
    print(f"stl: {time.perf_counter() - t0:g}")
    t0 = time.perf_counter()
    s = sort(keys, algo="radix_serial", num_bits=bits)
    print(f"serial radix: {time.perf_counter() - t0:g}")
    assert np.array_equal(s.numpy(), ref)
    t0 = time.perf_counter()
    p = sort(keys, algo="radix", num_bits=bits)
    print(f"parallel radix: {time.perf_counter() - t0:g}")
    assert np.array_equal(p.numpy(), ref)
    if gpu and torch.cuda.is_available():
        d = keys.cuda()
        sort(d)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g = sort(d)
        torch.cuda.synchronize()
        print(f"gpu radix: {time.perf_counter() - t0:g}")
        assert np.array_equal(g.cpu().numpy(), ref)
    return 0


def mergesort_main(argv=None) -> int:
    from ..ops.sort import merge_sort_cpu, sort

    argv = list(sys.argv[1:] if argv is None else argv)
    gpu = "--gpu" in argv
    argv = [x for x in argv if x != "--gpu"]
    if len(argv) != 4:
        print("order of arguments is: sortThreshold mergeThreshold numElementsToSort performSerialSort")
        print("setting performSerialSort to any non-zero value will perform std::sort and check for correctness of "
              "the merge sort")
        print("you will want to set this to 0 when you are doing tuning")
        return 1
    sort_thr, merge_thr, n, do_serial = (int(x) for x in argv)
    keys = torch.from_numpy(np.random.default_rng(0).integers(0, 2**31 - 1, n, dtype=np.int64).astype(np.int32))
    ref = None
    if do_serial:
        t0 = time.perf_counter()
        ref = np.sort(keys.numpy())
        print(f"STL sort took: {time.perf_counter() - t0:g}")
    t0 = time.perf_counter()
    out, _ = merge_sort_cpu(keys, sort_thr, merge_thr)
    print(f"Merge sort took: {time.perf_counter() - t0:g}")
    if ref is not None:
        assert np.array_equal(out.numpy(), ref)
    if gpu and torch.cuda.is_available():
        d = keys.cuda()
        sort(d, algo="merge")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g = sort(d, algo="merge")
        torch.cuda.synchronize()
        print(f"GPU merge sort took: {time.perf_counter() - t0:g}")
        if ref is not None:
            assert np.array_equal(g.cpu().numpy(), ref)
    return 0
