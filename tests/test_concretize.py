"""Keccak hash concretisation (mythril_amd/concretize.py) against the reference's
``_replace_with_actual_sha`` behaviour (mythril/analysis/solver.py:129-165), with the
oracle's Keccak-256 as the hasher on CPU and the GPU kernel in the gpu-marked test."""

import pyoracle as O
import pytest

from mythril_amd import concretize
from mythril_amd.keccak_manager import KeccakFunctionManager
from mythril_amd.smt import symbol_factory
from mythril_amd.smt.interp import Witness
from mythril_amd.smt.model import Model, WitnessModel
from mythril_amd.smt.to_dag import TermLowering, UFRegistry

BV = symbol_factory.BitVecSym


def _model_with(x_val):
    reg = UFRegistry()
    kfm = KeccakFunctionManager(reg)
    x = BV("x", 256)
    h = kfm.create_keccak(x)
    cs = [kfm.create_conditions().raw]
    lo = TermLowering(reg).lower(cs)
    vals = [x_val if t.op == "var" and t.val == "x" else 0 for t in lo.var_terms]
    w = Witness(lo, vals, reg)
    return kfm, Model([WitnessModel(w, cs)]), h


def _oracle_hasher(calls):
    def h(msgs):
        calls.append(len(msgs))
        return [O.keccak256(m) for m in msgs]
    return h


def _replace(x_val, inputs, hasher):
    kfm, model, h = _model_with(x_val)
    hv = model.eval(h.raw).as_long()
    assert hex(hv)[2:].startswith(concretize.HASH_MATCHER)   # the interval prefix
    txs = [{"input": s.format(h=f"{hv:064x}")} for s in inputs]
    concretize.replace_with_actual_sha(txs, model, kfm=kfm, hasher=hasher)
    return txs


def test_hash_in_calldata_is_replaced_by_real_keccak():
    calls = []
    txs = _replace(1234, ["0xa9059cbb{h}" + "00" * 32, "0x12345678" + "00" * 32], _oracle_hasher(calls))
    want = O.keccak256((1234).to_bytes(32, "big")).hex()
    assert txs[0]["input"] == "0xa9059cbb" + want + "00" * 32
    assert txs[1]["input"] == "0x12345678" + "00" * 32          # no matcher: untouched
    assert calls == [1]                                            # one batched launch


def test_repeated_hash_is_replaced_everywhere_with_one_batch():
    calls = []
    txs = _replace(7, ["0xdeadbeef{h}{h}", "0xdeadbeef{h}"], _oracle_hasher(calls))
    want = O.keccak256((7).to_bytes(32, "big")).hex()
    assert txs[0]["input"] == "0xdeadbeef" + want + want
    assert txs[1]["input"] == "0xdeadbeef" + want
    assert calls == [1]


@pytest.mark.gpu
def test_gpu_concretisation_and_code_hash(engine):
    txs = _replace(99, ["0xa9059cbb{h}"], concretize._batch_keccak)
    assert txs[0]["input"] == "0xa9059cbb" + O.keccak256((99).to_bytes(32, "big")).hex()
    code = "0x6080604052348015600f57600080fd5b50"
    assert concretize.get_code_hash(code) == "0x" + O.keccak256(bytes.fromhex(code[2:])).hex()
    assert concretize.code_hashes([code, "0x", "zz"]) == [
        "0x" + O.keccak256(bytes.fromhex(code[2:])).hex(), "0x" + O.keccak256(b"").hex(), ""]


def _live_scenario(monkeypatch, gpu_min):
    """The stand-in Mythril with the report's concretisation step (analysis/solver.py:96-99
    -> :129-165, restated in tests/mythril_standin.py) over the facade keccak manager."""
    import copy
    import sys
    import types

    import fake_z3
    import mythril_standin
    from mythril_amd import integration

    mythril_standin.install(monkeypatch, fake_z3)
    monkeypatch.setattr(concretize, "GPU_MIN", gpu_min)
    kfm, model, h = _model_with(4321)
    kfm2, model2, h2 = _model_with(77)
    mods = sys.modules
    monkeypatch.setattr(mods["mythril.laser.ethereum.function_managers"], "keccak_function_manager", kfm)
    monkeypatch.setattr(mods["mythril.laser.smt"], "symbol_factory", symbol_factory, raising=False)
    hv = model.eval(h.raw).as_long()
    code = types.SimpleNamespace(bytecode="6080604052" + f"{hv:064x}")
    inputs = ["0xa9059cbb" + f"{hv:064x}" + "00" * 32, "0x12345678" + "00" * 32,
              "0xdeadbeef" + f"{hv:064x}" * 2, "0x" + code.bytecode + f"{hv:064x}"]
    sol = mods["mythril.analysis.solver"]
    want = [{"input": s} for s in inputs]
    sol.get_transaction_sequence_tail(want, model)
    want_code = [{"input": inputs[3]}]
    sol.get_transaction_sequence_tail(want_code, model, code)
    integration.install()
    assert sol._replace_with_actual_sha is concretize.live_replace_with_actual_sha
    got = [{"input": s} for s in inputs]
    sol.get_transaction_sequence_tail(got, model)
    got_code = [{"input": inputs[3]}]
    sol.get_transaction_sequence_tail(got_code, model, code)
    assert got == want and got_code == want_code
    hx = O.keccak256((4321).to_bytes(32, "big")).hex()
    assert want[0]["input"] == "0xa9059cbb" + hx + "00" * 32
    assert want_code[0]["input"] == "0x" + code.bytecode + hx   # the code part is kept
    return got


@pytest.mark.parametrize("gpu_min", [1, 192])
def test_installed_concretisation_matches_the_reference(monkeypatch, gpu_min):
    """integration.install() rebinds mythril.analysis.solver._replace_with_actual_sha; the
    rebound function rewrites calldata exactly as the reference's does — on the batched
    kernel path (gpu_min 1; the oracle engine here) and on the host path (192)."""
    import oracle_engine

    oracle_engine.install(monkeypatch)
    _live_scenario(monkeypatch, gpu_min)


@pytest.mark.gpu
def test_gpu_installed_concretisation_matches_the_reference(monkeypatch, engine):
    _live_scenario(monkeypatch, 1)
