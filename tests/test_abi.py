"""CPU: the C ABI and its Python mirror agree; the library loads and exports every symbol."""

import ctypes
import os
import re
import subprocess

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
