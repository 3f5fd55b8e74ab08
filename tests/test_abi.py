"""The C-ABI boundary (include/pebble_amd.h) without a GPU: the in-tree library
loads, exports every function the header declares, reports the header's ABI
version, and the Python mirror's constants equal the header's #defines.
No compute call is made (pbl_decode_batch needs a device)."""
import ctypes
import os
import re

from pebble_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = open(os.path.join(ROOT, "include", "pebble_amd.h")).read()


def _declared_functions():
    body = re.sub(r"/\*.*?\*/", "", HDR, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w \*]*?\b(pbl_\w+)\s*\(", body, flags=re.M)))


def _defines():
    return {m.group(1): int(m.group(2), 0)
            for m in re.finditer(r"#define\s+(PBL_\w+)\s+(0x[0-9A-Fa-f]+|\d+)u?\b", HDR)}


def test_library_exports_every_declared_function():
    lib = ctypes.CDLL(N.LIB_PATH)
    fns = _declared_functions()
    assert "pbl_decode_batch" in fns and len(fns) >= 15
    missing = [f for f in fns if not hasattr(lib, f)]
    assert not missing, missing


def test_abi_version_matches_header():
    lib = ctypes.CDLL(N.LIB_PATH)
    lib.pbl_abi_version.restype = ctypes.c_int
    assert lib.pbl_abi_version() == _defines()["PBL_ABI_VERSION"]


def test_python_constants_match_header():
    d = _defines()
    checked = 0
    for name, v in d.items():
        if hasattr(N, name):
            assert getattr(N, name) == v, name
            checked += 1
    assert checked >= 8
    assert N.PBL_BATCH_VARLEN == d["PBL_BATCH_VARLEN"]


def test_ctypes_struct_layouts_match_library():
    """sizeof/offsetof of the ctypes mirrors equal the compiled library's
    (pbl_struct_layout), field by field."""
    L = N.lib()
    cap = 256
    buf = (ctypes.c_uint64 * cap)()
    n = L.pbl_struct_layout(ctypes.cast(buf, ctypes.c_void_p), cap)
    v = list(buf[:n])
    exp = []
    for S in (N.BlockBatchC, N.TotalsC, N.DecodeOutC, N.TransformsC, N.FooterC, N.IndexOutC, N.KvOutC,
              N.ValueOutC, N.KvC, N.KvMetaC):
        exp.append(ctypes.sizeof(S))
        exp += [getattr(S, f).offset for f, _ in S._fields_]
    assert v == exp


def test_every_declared_function_has_a_ctypes_signature():
    assert set(_declared_functions()) == set(N.SIGNATURES)
