"""hw3 Vigenere drivers (same argv / output files as the reference).

    python -m cme213x create_cipher <book> <period>      -> cipher_text.txt
    python -m cme213x solve_cipher <cipher_text.txt>     -> plain_text.txt
"""
from __future__ import annotations

import sys


def create_cipher_main(argv=None) -> int:
    from ..models.vigenere import create_cipher

    argv = sys.argv[1:] if argv is None else argv
    if len(argv) < 2:
        print("usage: create_cipher <book> <period>")
        return 1
    create_cipher(open(argv[0], "rb").read(), int(argv[1]))
    return 0


def solve_cipher_main(argv=None) -> int:
    from ..models.vigenere import solve_cipher

    argv = sys.argv[1:] if argv is None else argv
    if len(argv) < 1:
        print("usage: solve_cipher <cipher_text.txt>")
        return 1
    solve_cipher(open(argv[0], "rb").read())
    return 0
