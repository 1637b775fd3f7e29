"""CPU: the C ABI and its Python mirror agree; the library loads and exports every symbol."""

import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from mythril_amd import _lib, ir

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_enum():
    src = open(os.path.join(ROOT, "include", "pf_bytecode.h")).read()
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"\bPF_([A-Z0-9_]+)\s*=\s*(\d+)", src)}


def test_opcodes_match_header():
    h = _header_enum()
    for name, val in h.items():
        if name in ("NUM_OPCODES",) or name.startswith("VK_"):
            continue
        assert getattr(ir, name) == val, name
    for k in ("GENERIC", "ACTOR", "KECCAK", "SMALL", "BOOL"):
        assert getattr(ir, "VK_" + k) == h["VK_" + k]


def test_register_counts_match_header():
    src = open(os.path.join(ROOT, "include", "pf_bytecode.h")).read()
    assert int(re.search(r"#define PF_NW (\d+)", src).group(1)) == ir.NW
    assert int(re.search(r"#define PF_NB (\d+)", src).group(1)) == ir.NB


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "pathfeas.h")).read()
    return set(re.findall(r"^\s*(?:int|const char\*)\s+(pf_[a-z0-9_]+)\(", src, re.M))


def test_ctypes_table_covers_header():
    assert _declared_symbols() == set(_lib.SIGNATURES)


def test_library_loads_and_exports():
    if not os.path.exists(_lib.LIB_PATH):
        from mythril_amd.build import build_library
        build_library()
    L = _lib.load_library()
    for name in _declared_symbols():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True).stdout
    for name in _declared_symbols():
        assert re.search(rf"\bT {name}\b", out), name


def test_set_desc_layout():
    assert ctypes.sizeof(_lib.pf_stats) == 40


def test_library_loads_without_torch_when_asked():
    """PF_TORCH=0 (set by integration.install() for a Mythril analysis process): the engine
    library loads on /opt/rocm's HIP runtime without importing torch."""
    import subprocess
    import sys

    code = ("import sys; from mythril_amd import _lib; _lib.load_library(); "
            "print('torch' in sys.modules)")
    env = dict(os.environ, PF_TORCH="0")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "False"


@pytest.mark.gpu
def test_engine_runs_without_torch_on_gpu():
    """The analysis-process configuration on the device: PF_TORCH=0, the engine initialises
    on /opt/rocm's runtime alone, hashes and searches, and torch is never imported."""
    import subprocess
    import sys

    code = (
        "import sys\n"
        "from mythril_amd import synth\n"
        "from mythril_amd.engine import get_engine\n"
        "e = get_engine()\n"
        "h = e.keccak256([b''])[0].hex()\n"
        "assert h == 'c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470', h\n"
        "progs = [synth.random_dag_set(i)[0] for i in range(8)]\n"
        "r = e.check(e.upload(progs), budget=4096, seed=0, flags=2)\n"
        "assert (r.found == 0).all(), r.found\n"
        "print('torch' in sys.modules)\n")
    env = dict(os.environ, PF_TORCH="0")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.strip().splitlines()[-1] == "False"


def test_pointer_helpers_pass_the_buffer_address():
    """_lib.ptr_* and native_terms._p32/_p8/_pi8 hand ctypes the numpy buffer's own address
    (from_buffer, or data_as for read-only and empty arrays) and refuse non-contiguous
    arrays, as ndarray.ctypes.data_as with the contiguity assert did."""
    from mythril_amd.smt import native_terms as NT

    def addr(p):
        return ctypes.cast(p, ctypes.c_void_p).value

    a = np.arange(16, dtype=np.uint32)
    ro = np.frombuffer(np.arange(4, dtype=np.uint32).tobytes(), dtype=np.uint32)
    assert not ro.flags.writeable
    empty = np.zeros(0, dtype=np.uint32)
    for x in (a, ro, empty, a.reshape(4, 4)):
        assert addr(_lib.ptr_u32(x)) == x.ctypes.data or x.size == 0
        assert addr(NT._p32(x)) == x.ctypes.data or x.size == 0
    b = np.arange(8, dtype=np.uint8)
    assert addr(_lib.ptr_u8(b)) == b.ctypes.data and addr(NT._p8(b)) == b.ctypes.data
    c = np.arange(4, dtype=np.uint64)
    assert addr(_lib.ptr_u64(c)) == c.ctypes.data
    i8 = np.zeros(8, dtype=np.int8)
    assert addr(NT._pi8(i8)) == i8.ctypes.data
    with pytest.raises(AssertionError):
        _lib.ptr_u32(a[::2])
    with pytest.raises(AssertionError):
        _lib.ptr_u32(a.astype(np.int64))
    # a native call writes through the pointer into the array itself
    libc = ctypes.CDLL(None)
    libc.memset.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_int, ctypes.c_size_t]
    libc.memset(_lib.ptr_u32(a), 0, a.nbytes)
    assert not a.any()
