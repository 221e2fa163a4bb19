"""Incremental native build: a source is rebuilt when a header it reaches
through quoted #includes changes -- one next to it (csrc/hip/heat_pipe.h is
shared by the production and tuning sources of the pipelined heat pass) or
one under csrc/include/cme213/, transitively -- and only then."""
import importlib
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build():
    return importlib.import_module("2012-04_stanford_cme213_amd._build")


def test_includes_of_pipe_sources():
    b = _build()
    hip = b.CSRC / "hip"
    for src in (hip / "heat_pipe.hip", b.CSRC / "hip_tune" / "heat_pipe_tune.hip"):
        assert (hip / "heat_pipe.h").resolve() in b._includes(src), src
    inc = b._includes(hip / "heat2d.hip")
    assert (hip / "heat2d_kernels.h").resolve() in inc
    assert (b.INCLUDE / "cme213" / "common.h").resolve() in b._includes(hip / "heat2d_kernels.h")


def test_tuning_arms_are_not_in_the_production_library():
    """The tuning arms (pipelined-pass A/B instantiations, streaming-kernel
    and scan sweeps, the persistent dataflow and resident-tile schedules)
    build only with CME_TUNE=1, into libcme213_tune.so; the production
    library exports none of their entry points and stays under 13.8 MiB."""
    import ctypes

    b = _build()
    for f in ("heat_pipe_tune.hip", "heat_flow.hip", "heat_tile_res.hip"):
        assert not (b.CSRC / "hip" / f).exists(), f
    lib = ctypes.CDLL(str(b.HIP_LIB))
    for name in ("cme_heat_pipe_tune", "cme_heat_flow_f32", "cme_heat_tile_res_f32", "cme_heat_streamn_tune",
                 "cme_heat_stream2_tune", "cme_scan_tune", "cme_spmv_scan_tune"):
        assert not hasattr(lib, name), name
    assert hasattr(lib, "cme_heat_pipe_f32") and hasattr(lib, "cme_tune_set")
    assert b.HIP_LIB.stat().st_size <= 13.8 * 2 ** 20


def test_needs_rebuild_on_reached_header(tmp_path):
    b = _build()
    hdr = tmp_path / "k.h"
    inner = tmp_path / "inner.h"
    other = tmp_path / "other.h"
    src = tmp_path / "k.hip"
    obj = tmp_path / "k.o"
    inner.write_text("#pragma once\n")
    hdr.write_text('#pragma once\n#include "inner.h"\n')
    other.write_text("#pragma once\n")
    src.write_text('#include "k.h"\n')
    obj.write_text("")
    t = obj.stat().st_mtime
    for f in (hdr, inner, src, other):
        os.utime(f, (t - 10, t - 10))
    assert not b._needs(obj, src)
    os.utime(other, (t + 10, t + 10))  # not included: no rebuild
    assert not b._needs(obj, src)
    os.utime(inner, (t + 10, t + 10))  # reached through k.h
    assert b._needs(obj, src)
