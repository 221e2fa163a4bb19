"""Sorts (GPU radix/merge, OpenMP radix/merge) and the hw3 text pipeline."""
import os

import numpy as np
import pytest
import torch

from cme213x.models.vigenere import create_cipher, solve_cipher
from cme213x.ops.sort import merge_sort_cpu, sort
from cme213x.ops.text import (digraph_histogram, histogram_u8, letter_histogram, match_counts,
                              residue_histograms, sanitize, vigenere)

BOOK = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "mobydick_hw3.txt.gz")


# English letter frequencies (%), a..z: a synthetic corpus with the same
# statistics when the reference's moby dick is not mounted (e.g. GPU box).
_EN = [8.17, 1.49, 2.78, 4.25, 12.70, 2.23, 2.02, 6.09, 6.97, 0.15, 0.77, 4.03, 2.41, 6.75, 7.51, 1.93, 0.10,
       5.99, 6.33, 9.06, 2.76, 0.98, 2.36, 0.15, 1.97, 0.07]


def _book():
    if os.path.exists(BOOK):
        import gzip

        return gzip.open(BOOK, "rb").read()
    rng = np.random.default_rng(0)
    p = np.asarray(_EN) / sum(_EN)
    letters = rng.choice(np.arange(97, 123, dtype=np.uint8), size=1_200_000, p=p)
    caps = rng.random(letters.size) < 0.03
    letters[caps] -= 32  # some upper case, lowered by sanitize
    text = letters.astype(np.uint8)
    spaces = rng.random(text.size) < 0.18
    text[spaces] = ord(" ")  # non-letters removed by sanitize
    return text.tobytes()


@pytest.mark.parametrize("algo", ["radix", "radix_serial"])
@pytest.mark.parametrize("bits", [4, 8, 11, 16])
def test_cpu_radix(algo, bits):
    x = torch.randint(0, 2**31 - 1, (50001,), dtype=torch.int32)
    assert torch.equal(sort(x, algo=algo, num_bits=bits), torch.sort(x).values)


@pytest.mark.parametrize("thr", [(1, 2), (100, 100), (10000, 64)])
def test_cpu_merge(thr):
    x = torch.randint(-1000, 1000, (100003,), dtype=torch.int32)
    y, st = merge_sort_cpu(x, *thr)
    assert st in (1, -1) and torch.equal(y, torch.sort(x).values)


def test_text_pipeline_cpu():
    book = _book()
    clean = sanitize(torch.from_numpy(np.frombuffer(book, np.uint8).copy()))
    if os.path.exists(BOOK):
        assert clean.numel() == 967673  # hw3 writeup: sanitized moby dick length
        h = letter_histogram(clean).numpy() / clean.numel()
        assert abs(h[4] - 0.12294) < 1e-4  # 'e' frequency from the writeup
    c, key = create_cipher(book, 53, device="cpu", out_path=None)
    r = solve_cipher(c, device="cpu", out_path=None, verbose=False)
    assert r["key_length"] == 53 and np.array_equal(r["shifts"], key % 26)
    assert np.array_equal(r["plain"], clean.numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 1000, 4096, 100003, 3_000_001])
@pytest.mark.parametrize("dtype", [torch.int32, torch.float32])
@pytest.mark.parametrize("algo", ["radix", "merge"])
def test_gpu_sort_keys(gpu, n, dtype, algo):
    x = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32) if dtype == torch.int32 else torch.randn(n)
    y = sort(x.to(gpu), algo=algo).cpu()
    assert torch.equal(y, torch.sort(x).values)


@pytest.mark.gpu
def test_gpu_radix_key_value_stable(gpu):
    n = 1_000_003
    k = torch.randint(0, 1000, (n,), dtype=torch.int32)  # many duplicates
    v = torch.arange(n, dtype=torch.int32)
    ks, vs = sort(k.to(gpu), v.to(gpu), algo="radix")
    ref = torch.sort(k, stable=True)
    assert torch.equal(ks.cpu(), ref.values) and torch.equal(vs.cpu(), ref.indices.to(torch.int32))


@pytest.mark.gpu
def test_gpu_text_kernels(gpu):
    book = _book()
    raw = torch.from_numpy(np.frombuffer(book, np.uint8).copy())
    clean_c = sanitize(raw)
    clean_g = sanitize(raw.to(gpu))
    assert torch.equal(clean_g.cpu(), clean_c)
    assert torch.equal(histogram_u8(raw.to(gpu)).cpu(), histogram_u8(raw))
    assert torch.equal(letter_histogram(clean_g).cpu(), letter_histogram(clean_c))
    assert torch.equal(digraph_histogram(clean_g).cpu(), digraph_histogram(clean_c))
    for p in (7, 500, 3000):
        assert torch.equal(residue_histograms(clean_g, p).cpu(), residue_histograms(clean_c, p))
    small = clean_c[:200000]
    assert torch.equal(match_counts(small.to(gpu), 1, 50).cpu(), match_counts(small, 1, 50))
    assert torch.equal(match_counts(small.to(gpu), 1990, 40).cpu(), match_counts(small, 1990, 40))
    key = torch.randint(1, 26, (123,), dtype=torch.int32)
    enc = vigenere(clean_g, key)
    assert torch.equal(enc.cpu(), vigenere(clean_c, key))
    assert torch.equal(vigenere(enc, key, decode=True).cpu(), clean_c)


@pytest.mark.gpu
@pytest.mark.parametrize("period", [11, 500])
def test_gpu_vigenere_roundtrip(gpu, period):
    book = _book()
    c, key = create_cipher(book, period, device=gpu, out_path=None)
    r = solve_cipher(c, device=gpu, out_path=None, verbose=False)
    assert r["key_length"] == period and np.array_equal(r["shifts"], key % 26)
