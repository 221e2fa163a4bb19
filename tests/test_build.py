"""Incremental native build: a source is rebuilt when a header next to it
that it includes by quoted relative path changes (csrc/hip/heat_pipe.h is
shared by the production and tuning sources of the pipelined heat pass)."""
import importlib
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build():
    return importlib.import_module("2012-04_stanford_cme213_amd._build")


def test_local_includes_of_pipe_sources():
    b = _build()
    hip = b.CSRC / "hip"
    for src in (hip / "heat_pipe.hip", b.CSRC / "hip_tune" / "heat_pipe_tune.hip"):
        assert (hip / "heat_pipe.h").resolve() in b._local_includes(src), src
    # include-directory headers are tracked by the newest-header rule, not here
    assert all(h.parent == hip.resolve() for h in b._local_includes(hip / "heat2d.hip"))


def test_tuning_arms_are_not_in_the_production_library():
    """heat_pipe_tune (the pipelined pass's A/B arms) builds only with
    CME_TUNE=1, into libcme213_tune.so; the production library does not
    export its entry point."""
    import ctypes

    b = _build()
    assert not (b.CSRC / "hip" / "heat_pipe_tune.hip").exists()
    lib = ctypes.CDLL(str(b.HIP_LIB))
    assert not hasattr(lib, "cme_heat_pipe_tune")
    assert hasattr(lib, "cme_heat_pipe_f32") and hasattr(lib, "cme_tune_set")


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
