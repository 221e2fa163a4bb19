"""Incremental native build: a source is rebuilt when a header next to it
that it includes by quoted name changes (csrc/hip/heat_pipe.h is shared by
the production and tuning sources of the pipelined heat pass)."""
import importlib
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build():
    return importlib.import_module("2012-04_stanford_cme213_amd._build")


def test_local_includes_of_pipe_sources():
    b = _build()
    hip = b.CSRC / "hip"
    for src in ("heat_pipe.hip", "heat_pipe_tune.hip"):
        assert hip / "heat_pipe.h" in b._local_includes(hip / src), src
    # include-directory headers are tracked by the newest-header rule, not here
    assert all(h.parent == hip for h in b._local_includes(hip / "heat2d.hip"))


def test_needs_rebuild_on_local_header(tmp_path):
    b = _build()
    hdr = tmp_path / "k.h"
    src = tmp_path / "k.hip"
    obj = tmp_path / "k.o"
    hdr.write_text("#pragma once\n")
    src.write_text('#include "k.h"\n')
    obj.write_text("")
    t = obj.stat().st_mtime
    os.utime(hdr, (t - 10, t - 10))
    os.utime(src, (t - 10, t - 10))
    assert not b._needs(obj, src, 0.0)
    os.utime(hdr, (t + 10, t + 10))
    assert b._needs(obj, src, 0.0)
