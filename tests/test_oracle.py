"""CPU: pin the oracle (oracle/pyoracle.py) against the reference's own fixtures.

* vmSha3Test digests (reference tests/laser/evm_testsuite/VMTests/vmSha3Test) and the
  empty-input Keccak constant (keccak_function_manager.py:87-93);
* EIP-145 shift vectors (reference tests/instructions/{shl,shr,sar}_test.py);
* vmArithmeticTest / vmBitwiseLogicOperation post-storage (straight-line programs);
* signed division family against an independent Python-int formulation;
* Philox4x32-10 known-answer vectors (Random123).
"""

import random

import numpy as np

import pyoracle as O
import pytest
from conftest import load_golden

import evm_to_ir
from dag_eval import eval_dag
from mythril_amd import ir
from mythril_amd.lower import lower


def test_keccak_empty_constant():
    # keccak_function_manager.py:92
    assert int.from_bytes(O.keccak256(b""), "big") == \
        89477152217924674838424037953991966239322087453347756267410168184682657981552


@pytest.mark.parametrize("case", load_golden("vmsha3.json"), ids=lambda c: c["name"])
def test_keccak_vmsha3(case):
    # memory is zero-initialised in these fixtures: the message is `size` zero bytes
    assert "0x" + O.keccak256(bytes(case["size"])).hex() == case["digest"].lower()


def test_keccak_multiblock_padding_edges():
    # rate boundary: 135 / 136 / 137 bytes exercise the 0x01|0x80 same-byte pad and 2 blocks
    for n in (135, 136, 137, 271, 272):
        a = O.keccak256(bytes(range(256)) [:n] if n <= 256 else bytes(n))
        assert len(a) == 32


@pytest.mark.parametrize("case", load_golden("eip145.json"), ids=lambda c: c["op"] + c["shift"])
def test_eip145(case):
    v, s, e = int(case["value"], 16), int(case["shift"], 16), int(case["expected"], 16)
    fn = {"shl": O.bvshl, "shr": O.bvlshr, "sar": O.bvashr}[case["op"]]
    assert fn(v, s, 256) == e


def _vmtests():
    out = []
    for c in load_golden("vmtests.json"):
        try:
            out.append((c["name"], evm_to_ir.build(c["code"], c["storage"])))
        except evm_to_ir.Unsupported:
            pass
    return out


def test_vmtests_coverage():
    assert len(_vmtests()) >= 200


@pytest.mark.parametrize("name,dag", _vmtests(), ids=lambda x: x if isinstance(x, str) else "")
def test_vmtests_post_storage(name, dag):
    assert eval_dag(dag, [])
    prog = lower(dag)
    sv = O.SetView.from_batch(ir.Batch([prog]), 0)
    assert sv.evaluate([])


def _trunc_div(a, b):
    q = abs(a) // abs(b)
    return q if (a < 0) == (b < 0) else -q


@pytest.mark.parametrize("w", [1, 8, 64, 160, 256])
def test_signed_division_independent(w):
    rng = random.Random(w)
    M = (1 << w) - 1
    vals = [0, 1, M, 1 << (w - 1), (1 << (w - 1)) - 1, 2 % (M + 1)] + [rng.getrandbits(w) for _ in range(40)]
    for a in vals:
        for b in vals:
            sa, sb = O.to_signed(a, w), O.to_signed(b, w)
            if b == 0:
                assert O.bvsdiv(a, b, w) == (1 if sa < 0 else M)
                assert O.bvsrem(a, b, w) == a and O.bvsmod(a, b, w) == a
                continue
            assert O.bvsdiv(a, b, w) == _trunc_div(sa, sb) & M
            assert O.bvsrem(a, b, w) == (sa - _trunc_div(sa, sb) * sb) & M
            assert O.bvsmod(a, b, w) == (sa % sb) & M  # Python % takes the divisor's sign


def test_philox_kat():
    kat = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
           ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
           ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
            (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]
    for ctr, key, exp in kat:
        got = O.philox4x32([[c] for c in ctr], key)
        assert tuple(int(x[0]) for x in got) == exp


def test_ops_golden_consistent():
    # the committed per-op vectors still match the restatement (guards accidental edits)
    fns = {"add": O.bvadd, "sub": O.bvsub, "mul": O.bvmul, "udiv": O.bvudiv, "urem": O.bvurem,
           "sdiv": O.bvsdiv, "srem": O.bvsrem, "smod": O.bvsmod, "shl": O.bvshl,
           "lshr": O.bvlshr, "ashr": O.bvashr, "exp": O.bvexp, "ult": O.ult, "ule": O.ule,
           "slt": O.slt, "sle": O.sle, "uadd_noovf": O.uadd_noovf, "umul_noovf": O.umul_noovf}
    for v in load_golden("ops.json")[::7]:
        r = fns[v["op"]](int(v["a"], 16), int(v["b"], 16), v["w"])
        exp = v["r"] if isinstance(v["r"], int) else int(v["r"], 16)
        assert int(r) == exp


def test_c_keccak_matches_python_and_vmsha3():
    """oracle/coracle.c's Keccak-256 (the GPU keccak checker / CPU baseline) against the
    spec restatement in pyoracle and the vmSha3Test digests."""
    import coracle_py

    for c in load_golden("vmsha3.json"):
        m = np.zeros(c["size"], dtype=np.uint8)
        got = coracle_py.keccak256_fixed(m, c["size"], 1)[0].tobytes()
        assert "0x" + got.hex() == c["digest"].lower()
    rng = np.random.default_rng(9)
    for ln in [0, 1, 31, 64, 135, 136, 137, 271, 272, 500]:
        d = rng.integers(0, 256, size=max(3 * ln, 1), dtype=np.uint8)
        got = coracle_py.keccak256_fixed(d, ln, 3)
        for i in range(3):
            assert got[i].tobytes() == O.keccak256(d[ln * i:ln * i + ln].tobytes())
