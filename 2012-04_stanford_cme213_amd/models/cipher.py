"""hw1 part 1: Caesar shift cipher driver and the bandwidth sweeps.

Parity with ``hw/hw1/programming/cipher.cu:127-282``: read the book, replicate
it 16x (~19.76 MB), time H2D, run the CPU reference, run every lane width
(char / uint / uint2 and -- new on CDNA -- uint4), byte-exact check, write
``mobydick_enciphered.txt`` (original length). Sweeps: vector length
(``analysis/cipher_vl.cu:154-163``) and block size (``analysis/cipher_bs.cu:
156-170``) emitting CSV rows.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops.elementwise import shift_cipher
from ..utils.timer import EventTimer

SHIFT = 3  # default for the sweeps; the driver draws (rand() % 25) + 1 like cipher.cu:180


def load_text(path: str) -> np.ndarray:
    return np.fromfile(path, dtype=np.uint8)


def run_hw1_cipher(path: str, replicate: int = 16, shift: int | None = None, device: str | None = None,
                   out_path: str = "mobydick_enciphered.txt", seed: int = 0) -> dict:
    device = device or ("cuda" if torch.cuda.is_available() else "cpu")
    if shift is None:
        shift = int(np.random.default_rng(seed).integers(0, 25)) + 1  # never 0
    text = load_text(path)
    orig_len = text.size
    data = np.tile(text, replicate)
    host = torch.from_numpy(data)
    res = {"bytes": int(data.size), "shift": shift, "variants": {}}
    shift_cipher(host[:4096], shift)  # CPU warm-up (OpenMP thread start-up, library load)
    if device == "cpu":
        t = EventTimer("host shift cypher")
        with t:
            ref = shift_cipher(host, shift)
        res["cpu_ms"] = t.ms
        ref.numpy()[:orig_len].tofile(out_path)
        return res
    dev = torch.device(device)
    d_in = torch.empty_like(host, device=dev)
    # warm-up copies (reference :185-187)
    d_in.copy_(host)
    torch.cuda.synchronize()
    pinned = host.pin_memory()
    t = EventTimer("copy to gpu", device=dev)
    with t:
        d_in.copy_(pinned, non_blocking=True)
    res["h2d_ms"] = t.ms
    t = EventTimer("host shift cypher")
    with t:
        ref = shift_cipher(host, shift)
    res["cpu_ms"] = t.ms
    ref_np = ref.numpy()
    ok = True
    for name in ("char", "uint", "uint2", "uint4"):
        d_out = torch.empty_like(d_in)
        shift_cipher(d_in, shift, d_out, width=name)  # warm-up
        t = EventTimer(f"gpu shift cypher {name}", device=dev)
        with t:
            shift_cipher(d_in, shift, d_out, width=name)
        gpu = d_out.cpu().numpy()
        bad = np.flatnonzero(gpu != ref_np)
        if bad.size:
            ok = False
            print(f"{name}: first mismatch at {bad[0]}: {gpu[bad[0]]} != {ref_np[bad[0]]}")
        res["variants"][name] = {"ms": t.ms, "GBps_rw": 2 * data.size / t.ms / 1e6, "ok": not bad.size}
    # library baseline: the solution's thrust::transform(in, constant_iterator
    # (shift), plus<uchar>) (hw/hw1/solution/cipher_solution.cu:234-245) -> a
    # framework elementwise op (torch's uint8 add wraps mod 256 like uchar)
    d_out = torch.add(d_in, shift)
    t = EventTimer("gpu shift cypher library (torch.add)", device=dev)
    with t:
        torch.add(d_in, shift, out=d_out)
    lib = d_out.cpu().numpy()
    lib_ok = bool(np.array_equal(lib, ref_np))
    ok = ok and lib_ok
    res["variants"]["library"] = {"ms": t.ms, "GBps_rw": 2 * data.size / t.ms / 1e6, "ok": lib_ok}
    # device -> host of the result (reference PA1 section 1c reports both directions)
    pinned_out = torch.empty_like(pinned).pin_memory()
    t = EventTimer("copy from gpu", device=dev)
    with t:
        pinned_out.copy_(d_out, non_blocking=True)
    res["d2h_ms"] = t.ms
    res["h2d_GBps"] = data.size / res["h2d_ms"] / 1e6
    res["d2h_GBps"] = data.size / res["d2h_ms"] / 1e6
    if ok:
        print("All CUDA Versions matched reference output.  Outputting ciphered text.")
        ref_np[:orig_len].tofile(out_path)
    res["ok"] = ok
    return res


def sweep_vector_length(path: str, max_copies: int = 66, step: int = 1, widths=("char", "uint", "uint2", "uint4"),
                        device="cuda", shift: int = SHIFT) -> list[dict]:
    """Bandwidth vs vector length (CSV rows: bytes, GB/s per width; bytes/time,
    the spreadsheet convention of analysis/data_bandwidth_vector_length.csv)."""
    text = load_text(path)
    rows = []
    dev = torch.device(device)
    for k in range(16, max_copies + 1, step):
        d_in = torch.from_numpy(np.tile(text, k)).to(dev)
        d_out = torch.empty_like(d_in)
        row = {"bytes": int(d_in.numel())}
        for w in widths:
            shift_cipher(d_in, shift, d_out, width=w)
            t = EventTimer(w, device=dev, print_result=False)
            with t:
                shift_cipher(d_in, shift, d_out, width=w)
            row[w] = d_in.numel() / t.ms / 1e6
        rows.append(row)
    return rows


def sweep_block_size(path: str, widths=("char", "uint", "uint2", "uint4"), device="cuda",
                     shift: int = SHIFT) -> list[dict]:
    """Bandwidth vs block size. Wave64 means multiples of 64 are the meaningful
    points on CDNA (the reference swept 4..512 for 32-wide warps)."""
    text = np.tile(load_text(path), 16)
    dev = torch.device(device)
    d_in = torch.from_numpy(text).to(dev)
    d_out = torch.empty_like(d_in)
    rows = []
    for bs in (64, 128, 192, 256, 320, 384, 448, 512, 640, 768, 896, 1024):
        row = {"block": bs}
        for w in widths:
            shift_cipher(d_in, shift, d_out, width=w, block=bs)
            t = EventTimer(w, device=dev, print_result=False)
            with t:
                shift_cipher(d_in, shift, d_out, width=w, block=bs)
            row[w] = d_in.numel() / t.ms / 1e6
        rows.append(row)
    return rows
