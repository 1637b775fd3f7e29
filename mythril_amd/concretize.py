"""Keccak hash concretisation on the GPU — SURVEY §8(f) row 2.

When Mythril turns a model into a concrete transaction sequence it replaces every keccak
UF output that leaked into calldata (a value from the ``hash_matcher`` interval of the
keccak function manager) by the real Keccak-256 of the UF input the model assigns
(``_replace_with_actual_sha``, mythril/analysis/solver.py:129-165), and it hashes contract
code for CREATE2 / EXTCODEHASH (``get_code_hash``, mythril/support/support_utils.py:74-90).
The reference hashes one value at a time with eth_hash on the host.  Here every hash a
sequence needs is computed in ONE batched launch of the Keccak kernel
(``pf_keccak256_batch``): the candidate inputs are collected from the transactions first,
hashed together, and the reference's sequential replacement loop then runs against that
table (a value the prefetch did not anticipate — a window created by an earlier
replacement — is hashed on demand), so the output string is identical to the reference's.
"""

from __future__ import annotations

import os
from functools import lru_cache
from typing import Callable, Dict, List, Optional, Sequence

from .keccak_manager import KeccakFunctionManager, keccak_function_manager
from .smt import symbol_factory

HASH_MATCHER = "fffffff"   # keccak_function_manager.py:36, the interval prefix in hex


def _batch_keccak(messages: Sequence[bytes]) -> List[bytes]:
    from .engine import get_engine

    return get_engine().keccak256(list(messages))


def get_concrete_hash_data(kfm, model) -> Dict[int, List[int]]:
    """keccak_function_manager.py:132-148: model values of every symbolic hash, by size (the
    manager's own method: Mythril's or the mirror's)."""
    return kfm.get_concrete_hash_data(model)


def replace_with_actual_sha(concrete_transactions: List[Dict[str, str]], model, code=None,
                            kfm: Optional[KeccakFunctionManager] = None,
                            hasher: Callable[[Sequence[bytes]], List[bytes]] = _batch_keccak,
                            bvv=None) -> None:
    """Mirror of ``_replace_with_actual_sha`` (analysis/solver.py:129-165), batched.  ``kfm``
    and ``bvv`` (the ``BitVecVal`` constructor its functions take) default to this package's
    facade; the live seam passes Mythril's own (:func:`live_replace_with_actual_sha`)."""
    kfm = kfm or keccak_function_manager
    bvv = bvv or symbol_factory.BitVecVal
    concrete_hashes = get_concrete_hash_data(kfm, model)
    inverse_of = {}

    def preimage(value: int):
        """(size, input value) the model assigns to keccak^-1(value), as the reference's
        size loop does (the last matching size wins)."""
        if value in inverse_of:
            return inverse_of[value]
        res = None
        for size in concrete_hashes:
            if value not in concrete_hashes[size]:
                continue
            _, inverse = kfm.store_function[size]
            arg = bvv(value, 256)
            res = (size, model.eval(inverse(arg).raw).as_long() & ((1 << size) - 1))
        inverse_of[value] = res
        return res

    def msg(pre) -> bytes:
        size, v = pre
        return v.to_bytes(size // 8, "big")

    # 1. prefetch: every window of the original inputs that can be replaced, one launch
    table: Dict[bytes, bytes] = {}
    wanted = []
    for tx in concrete_transactions:
        inp = tx["input"]
        if HASH_MATCHER not in inp:
            continue
        s_index = len(code.bytecode) + 2 if code is not None and code.bytecode in inp else 10
        for i in range(s_index, len(inp)):
            window = inp[i:i + 64]
            if HASH_MATCHER not in window or len(window) != 64:
                continue
            pre = preimage(int(window, 16))
            if pre is not None and msg(pre) not in table:
                table[msg(pre)] = b""
                wanted.append(msg(pre))
    if wanted:
        for m, h in zip(wanted, hasher(wanted)):
            table[m] = h

    # 2. the reference's replacement loop, verbatim in behaviour
    for tx in concrete_transactions:
        if HASH_MATCHER not in tx["input"]:
            continue
        if code is not None and code.bytecode in tx["input"]:
            s_index = len(code.bytecode) + 2
        else:
            s_index = 10
        for i in range(s_index, len(tx["input"])):
            data_slice = tx["input"][i:i + 64]
            if HASH_MATCHER not in data_slice or len(data_slice) != 64:
                continue
            pre = preimage(int(data_slice, 16))
            if pre is None:
                continue
            m = msg(pre)
            if not table.get(m):
                table[m] = hasher([m])[0]
            hex_keccak = table[m].hex().rjust(64, "0")
            tx["input"] = tx["input"][:s_index] + tx["input"][s_index:].replace(
                tx["input"][i:64 + i], hex_keccak)


# preimages per call from which the GPU kernel hashes them (one launch); fewer go to the host
# Keccak Mythril already uses (eth_hash through support_utils.sha3, keccak_function_manager.py:
# 57-69): a launch costs tens of microseconds, eth_hash one or two per 64-byte message
# (profiles/r05j_keccak_latency.json: 43 us per launch against 0.4 us per message on the
# host, so the launch wins from ~200 messages on)
GPU_MIN = int(os.environ.get("PF_KECCAK_GPU_MIN", "192"))


def live_replace_with_actual_sha(concrete_transactions: List[Dict[str, str]], model, code=None) -> None:
    """The drop-in for ``mythril.analysis.solver._replace_with_actual_sha`` (installed by
    integration.install): the batched concretisation over Mythril's own keccak function
    manager and ``symbol_factory``; the preimages of a call are hashed in one GPU launch
    when there are ``GPU_MIN`` or more of them, else by Mythril's host ``sha3``."""
    from mythril.laser.ethereum.function_managers import keccak_function_manager as kfm
    from mythril.laser.smt import symbol_factory as sf
    from mythril.support.support_utils import sha3

    def hasher(msgs: Sequence[bytes]) -> List[bytes]:
        if len(msgs) >= GPU_MIN:
            return _batch_keccak(msgs)
        return [bytes(sha3(m)) for m in msgs]

    replace_with_actual_sha(concrete_transactions, model, code, kfm=kfm, hasher=hasher, bvv=sf.BitVecVal)


@lru_cache(maxsize=2 ** 10)
def get_code_hash(code) -> str:
    """Mirror of support_utils.get_code_hash (:74-90) on the GPU Keccak kernel."""
    if isinstance(code, tuple):
        return str(hash(code))
    code = code[2:] if code.startswith("0x") else code
    try:
        data = bytes.fromhex(code)
    except ValueError:
        return ""
    return "0x" + _batch_keccak([data])[0].hex()


def code_hashes(codes: Sequence[str]) -> List[str]:
    """Many code hashes in one launch (e.g. every account of a world state)."""
    blobs, idx = [], []
    out: List[str] = []
    for c in codes:
        c2 = c[2:] if c.startswith("0x") else c
        try:
            blobs.append(bytes.fromhex(c2))
            idx.append(len(out))
            out.append("")
        except ValueError:
            out.append("")
    for k, h in zip(idx, _batch_keccak(blobs) if blobs else []):
        out[k] = "0x" + h.hex()
    return out
