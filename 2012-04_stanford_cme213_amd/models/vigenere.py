"""hw3: Vigenere cipher -- create_cipher and solve_cipher drivers.

create (``hw/hw3/solution/create_cipher_solution.cu``): sanitize the book
(lowercase, keep a-z), draw a key of ``period`` shifts in 1..25, shift
periodically, write ``cipher_text.txt``.

solve (``hw/hw3/solution/solve_cipher_solution.cu``): letter frequencies,
top-20 digraphs of the non-overlapping pairs, key length by the kappa index of
coincidence ``ioc(i) = matches(i) / ((n-1)/26)`` -- the first i with ioc > 1.6
is the key length, confirmed when 2i also exceeds it -- then per-residue
frequency analysis (most frequent letter -> 'e'), decode, write
``plain_text.txt``. All analytics run as GPU kernels; the IOC is evaluated for
a batch of 1024 shifts per launch instead of one ``inner_product`` per shift.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops.text import (digraph_histogram, letter_histogram, match_counts, residue_histograms, sanitize,
                        vigenere)


def _dev(device):
    return torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))


def make_key(period: int, seed: int = 123) -> np.ndarray:
    """``period`` shifts uniform in 1..25 (never 0), seeded (the reference
    seeds its engine with 123; the exact engine sequence is not reproduced)."""
    return np.random.default_rng(seed).integers(1, 26, size=period).astype(np.int32)


def create_cipher(book: bytes | np.ndarray, period: int, seed: int = 123, device=None,
                  out_path: str | None = "cipher_text.txt") -> tuple[np.ndarray, np.ndarray]:
    dev = _dev(device)
    raw = torch.from_numpy(np.frombuffer(book, dtype=np.uint8).copy() if isinstance(book, bytes) else book).to(dev)
    clean = sanitize(raw)
    key = make_key(period, seed)
    cipher = vigenere(clean, torch.from_numpy(key)).cpu().numpy()
    if out_path:
        cipher.tofile(out_path)
    return cipher, key


def find_key_length(text: torch.Tensor, threshold: float = 1.6, batch: int = 1024, max_len: int = 100000,
                    verbose: bool = True) -> int:
    n = text.numel()
    norm = (n - 1) / 26.0
    key_len = 0
    s0 = 1
    while s0 < min(max_len, n):
        ns = min(batch, n - s0)
        ioc = match_counts(text, s0, ns).cpu().numpy() / norm
        for k, v in enumerate(ioc):
            i = s0 + k
            if verbose:
                print(f"Ioc: {v:g}")
            if v > threshold:
                if key_len == 0:
                    key_len = i
                elif i == 2 * key_len:
                    return key_len
                else:
                    raise RuntimeError("Unusual pattern in text!")
        s0 += ns
    raise RuntimeError("key length not found")


def solve_cipher(cipher: bytes | np.ndarray, device=None, out_path: str | None = "plain_text.txt",
                 verbose: bool = True) -> dict:
    dev = _dev(device)
    t = torch.from_numpy(np.frombuffer(cipher, dtype=np.uint8).copy() if isinstance(cipher, bytes) else cipher).to(dev)
    n = t.numel()
    hist = letter_histogram(t).cpu().numpy()
    if verbose:
        for i in range(26):
            print(f"{chr(97 + i)} {hist[i] / n:g}")
    dg = digraph_histogram(t).cpu().numpy().ravel()
    order = np.argsort(-dg, kind="stable")[:20]
    npairs = n // 2
    if verbose:
        for i in order:
            print(f"{chr(97 + i // 26)}{chr(97 + i % 26)} {dg[i] / npairs:g}")
    key_len = find_key_length(t, verbose=verbose)
    if verbose:
        print(f"keyLength: {key_len}")
    rh = residue_histograms(t, key_len).cpu().numpy()
    shifts = (np.argmax(rh, axis=1) - 4).astype(np.int32)  # most frequent letter -> 'e'
    plain = vigenere(t, torch.from_numpy(shifts), decode=True).cpu().numpy()
    if out_path:
        plain.tofile(out_path)
    return {"key_length": key_len, "shifts": shifts % 26, "plain": plain,
            "letter_freq": hist / n, "top_digraphs": [(chr(97 + i // 26) + chr(97 + i % 26), dg[i] / npairs)
                                                      for i in order]}
