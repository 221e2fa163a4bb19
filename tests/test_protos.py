"""Every ctypes prototype registered by the Python ops must match the C
signature of the exported native function (arity AND argument kinds): a
mismatch would pass garbage to a kernel launcher."""
import glob
import os
import re

import cme213x
from cme213x import _ext

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _kind(arg: str) -> str:
    a = " ".join(arg.replace("__restrict__", "").split())
    if a.startswith("const char*") or a.startswith("const char *"):
        return "s"
    if "*" in a:
        return "p"
    t = a.rsplit(" ", 1)[0] if " " in a else a
    return {"int": "i", "unsigned": "u", "uint32_t": "u", "long long": "q", "int64_t": "q", "float": "f",
            "double": "d", "unsigned long long": "Q", "uint64_t": "Q"}[t]


def _exports():
    sigs = {}
    for path in glob.glob(os.path.join(REPO, "csrc", "*", "*.*")):
        src = open(path).read()
        for m in re.finditer(r"CME(?:_CPU)?_EXPORT\s+[\w\s\*]+?\b(\w+)\s*\(([^)]*)\)", src):
            name, args = m.group(1), m.group(2)
            args = [a.strip() for a in args.split(",") if a.strip()]
            sigs[name] = "".join(_kind(a) for a in args)
    return sigs


def test_prototypes_match_native_signatures():
    import cme213x.ops  # noqa: F401  (registers every prototype)

    sigs = _exports()
    checked = 0
    for table in (_ext.HIP_PROTOS, _ext.CPU_PROTOS):
        for name, sig in table.items():
            assert name in sigs, f"{name}: no exported native function"
            assert sig.replace(" ", "") == sigs[name], f"{name}: proto {sig} != native {sigs[name]}"
            checked += 1
    assert checked > 20


def test_dist_abi_matches_ctypes_mirrors():
    """The ctypes mirrors of SubDesc / IpcPlan / IpcPeerDesc must have the
    native layout: the native loop reads them field by field."""
    import ctypes

    from cme213x.models.heat2d_dist import IpcPeerDesc, IpcPlan, SubDesc

    _ext.proto(_ext.HIP_PROTOS, "cme_dist_abi", "p")
    out = (ctypes.c_longlong * 5)()
    _ext.call_hip("cme_dist_abi", ctypes.addressof(out))
    assert list(out) == [ctypes.sizeof(SubDesc), SubDesc.ipc.offset, ctypes.sizeof(IpcPeerDesc),
                         ctypes.sizeof(IpcPlan), IpcPlan.peer.offset]
