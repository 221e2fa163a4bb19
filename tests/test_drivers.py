"""The command-line programs keep the reference's argv, stdout lines and
output files (CPU runs)."""
import os

import numpy as np
import pytest

from cme213x.__main__ import main


@pytest.fixture
def in_tmp(tmp_path):
    old = os.getcwd()
    os.chdir(tmp_path)
    yield tmp_path
    os.chdir(old)


def test_heat2d_mpi_loopback(in_tmp, capsys):
    with open("params.in", "w") as f:
        f.write("60 40\n1 1\n1\n5\n4\n5\n2\n0\n0 10 0 10\n")
    assert main(["heat2d_mpi", "params.in", "--ranks", "4", "--device", "cpu"]) == 0
    out = capsys.readouterr().out
    assert "5 iterations on a 60 by 40 grid took:" in out
    assert all(os.path.exists(f"grid{r}_final.txt") for r in range(4))


def test_heat2d_mpi_fast_arithmetic(in_tmp, capsys):
    """--fast (reassociated stencil, fp32, order 8) runs through the driver
    (bitwise equality of the decomposed run: test_heat_fast.py); other
    orders / fp64 are refused."""
    with open("params.in", "w") as f:
        f.write("60 72\n1 1\n1\n6\n8\n5\n1\n0\n0 10 0 10\n")
    assert main(["heat2d_mpi", "params.in", "--ranks", "4", "--device", "cpu", "--float", "--fast"]) == 0
    assert "6 iterations on a 60 by 72 grid took:" in capsys.readouterr().out
    assert all(os.path.exists(f"grid{r}_final.txt") for r in range(4))
    with open("params.in", "w") as f:
        f.write("60 72\n1 1\n1\n6\n4\n5\n1\n0\n0 10 0 10\n")
    with pytest.raises(ValueError, match="fast"):
        main(["heat2d_mpi", "params.in", "--ranks", "2", "--device", "cpu", "--float", "--fast", "--tblock", "2"])


def test_heat2d_cpu(in_tmp):
    with open("params.in", "w") as f:
        f.write("50 30\n1 1\n1\n3\n8\n5\n0 10 0 10\n")
    assert main(["heat2d", "params.in", "--device", "cpu"]) == 0
    assert os.path.exists("grid_init.txt") and os.path.exists("grid_final_cpu.txt")


def test_vigenere_cli(in_tmp):
    rng = np.random.default_rng(0)
    en = np.array([8.17, 1.49, 2.78, 4.25, 12.70, 2.23, 2.02, 6.09, 6.97, 0.15, 0.77, 4.03, 2.41, 6.75, 7.51, 1.93,
                   0.10, 5.99, 6.33, 9.06, 2.76, 0.98, 2.36, 0.15, 1.97, 0.07])
    rng.choice(np.arange(97, 123, dtype=np.uint8), 300000, p=en / en.sum()).tofile("book.txt")
    assert main(["create_cipher", "book.txt", "17"]) == 0
    assert main(["solve_cipher", "cipher_text.txt"]) == 0
    assert open("plain_text.txt", "rb").read() == open("book.txt", "rb").read()


def test_sort_clis(in_tmp, capsys):
    assert main(["radixsort", "20000", "8"]) == 0
    assert main(["mergesort", "64", "64", "20000", "1"]) == 0
    out = capsys.readouterr().out
    assert "parallel radix:" in out and "Merge sort took:" in out


def test_final_project_clis(in_tmp, capsys):
    assert main(["genfp", "3000", "200", "fpd", "--iters", "3"]) == 0
    assert main(["fp", "fpd/a.txt", "fpd/x.txt", "1"]) == 0
    assert main(["checker", "fpd/a.txt", "fpd/x.txt", "b.txt"]) == 0
    out = capsys.readouterr().out
    assert "The running time of my code for 3 iterations is:" in out
    assert "Relative L2 error" in out


def test_readmm(in_tmp):
    from cme213x.utils.mmio import read_matrix_market, write_matrix_market

    write_matrix_market("m.mtx", [0, 1, 2, 2], [0, 1, 0, 2], [1.0, 2.0, 3.0, 4.0], (3, 3))
    r, c, v, shape = read_matrix_market("m.mtx")
    assert shape == (3, 3) and v.tolist() == [1.0, 2.0, 3.0, 4.0]
    assert main(["readmm", "m.mtx", "out", "10", "2"]) == 0
    assert os.path.exists("out/a.txt")
