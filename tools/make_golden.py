#!/usr/bin/env python3
"""Extract the reference's own test DATA into tests/golden/ (run in the build container only).

Reads, as data, from /root/reference (never at test time — the GPU box has no reference):
  * tests/laser/evm_testsuite/VMTests/{vmArithmeticTest,vmBitwiseLogicOperation}/*.json —
    straight-line programs (PUSH/arith/SSTORE) and their expected post-storage
  * tests/laser/evm_testsuite/VMTests/vmSha3Test/*.json — SHA3 of zero memory and the digest
  * tests/instructions/{shl,shr,sar}_test.py — the EIP-145 (value, shift, expected) vectors
Writes tests/golden/{vmtests,vmsha3,eip145}.json.  Also writes tests/golden/ops.json: seeded
per-op vectors at widths {1, 8, 160, 255, 256} (boundary + random), whose expected values
come from oracle/pyoracle.py (the restatement — "parity unpinned" for z3-only corners).
"""

import json
import os
import random
import re
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
GOLD = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(REPO, "oracle"))

STRAIGHT = set(range(0x01, 0x0C)) | set(range(0x10, 0x1E)) | {0x50, 0x55} | set(range(0x60, 0xA0))
STRAIGHT |= {0x00}  # STOP


def opcodes(code_hex):
    b = bytes.fromhex(code_hex[2:])
    i, out = 0, []
    while i < len(b):
        o = b[i]
        out.append(o)
        if 0x60 <= o <= 0x7F:
            i += o - 0x5F
        i += 1
    return out


def vmtests():
    out = []
    for d in ("vmArithmeticTest", "vmBitwiseLogicOperation"):
        base = os.path.join(REF, "tests/laser/evm_testsuite/VMTests", d)
        for f in sorted(os.listdir(base)):
            j = json.load(open(os.path.join(base, f)))
            name, t = next(iter(j.items()))
            if "post" not in t:
                continue
            code = t["exec"]["code"]
            ops = opcodes(code)
            if not set(ops) <= STRAIGHT:
                continue
            addr = t["exec"]["address"]
            post = t["post"].get(addr, {}).get("storage", {})
            out.append({"suite": d, "name": name, "code": code, "storage": post})
    return out


def vmsha3():
    out = []
    base = os.path.join(REF, "tests/laser/evm_testsuite/VMTests/vmSha3Test")
    for f in sorted(os.listdir(base)):
        j = json.load(open(os.path.join(base, f)))
        name, t = next(iter(j.items()))
        if "post" not in t:
            continue
        code = bytes.fromhex(t["exec"]["code"][2:])
        # PUSHn size, PUSHm offset, SHA3 (0x20), PUSH1 0, SSTORE
        ops = opcodes(t["exec"]["code"])
        if ops[:3] not in ([0x60 + (code[0] - 0x60), None, 0x20],) and 0x20 not in ops:
            continue
        i, stack = 0, []
        while i < len(code):
            o = code[i]
            if 0x60 <= o <= 0x7F:
                n = o - 0x5F
                stack.append(int.from_bytes(code[i + 1:i + 1 + n], "big"))
                i += n + 1
                continue
            if o == 0x20:
                off, size = stack.pop(), stack.pop()
                stack.append(("sha3", off, size))
            elif o == 0x55:
                key, val = stack.pop(), stack.pop()
                if isinstance(val, tuple):
                    addr = t["exec"]["address"]
                    post = t["post"].get(addr, {}).get("storage", {})
                    exp = post.get(hex(key)) or post.get("0x%02x" % key)
                    if exp is not None and val[2] < 1 << 20:
                        out.append({"name": name, "offset": val[1], "size": val[2], "digest": exp})
            i += 1
    return out


def eip145():
    out = []
    for op in ("shl", "shr", "sar"):
        src = open(os.path.join(REF, "tests/instructions", f"{op}_test.py")).read()
        # the parametrised EIP-145 block: triples of hex strings
        trip = re.findall(r'\(\s*"(0x[0-9a-fA-F]+)",\s*"(0x[0-9a-fA-F]+)",\s*"(0x[0-9a-fA-F]+)",?\s*\)', src)
        for v, s, e in trip:
            out.append({"op": op, "value": v, "shift": s, "expected": e})
    return out


def ops_vectors(seed=20260101):
    import pyoracle as O
    rng = random.Random(seed)
    names = {
        "add": O.bvadd, "sub": O.bvsub, "mul": O.bvmul, "udiv": O.bvudiv, "urem": O.bvurem,
        "sdiv": O.bvsdiv, "srem": O.bvsrem, "smod": O.bvsmod, "shl": O.bvshl, "lshr": O.bvlshr,
        "ashr": O.bvashr, "exp": O.bvexp, "ult": O.ult, "ule": O.ule, "slt": O.slt, "sle": O.sle,
        "uadd_noovf": O.uadd_noovf, "umul_noovf": O.umul_noovf,
    }
    out = []
    for w in (1, 8, 160, 255, 256):
        M = (1 << w) - 1
        pool = [0, 1, 2, M, M - 1, 1 << (w - 1), (1 << (w - 1)) - 1, w, w - 1, w + 1]
        pool = sorted({p & M for p in pool})
        for name, fn in names.items():
            pairs = [(a, b) for a in pool for b in pool]
            pairs += [(rng.getrandbits(w), rng.getrandbits(w)) for _ in range(24)]
            pairs += [(rng.getrandbits(w), rng.getrandbits(min(w, 9))) for _ in range(8)]
            for a, b in pairs:
                r = fn(a, b, w)
                out.append({"op": name, "w": w, "a": hex(a), "b": hex(b),
                            "r": (int(r) if isinstance(r, bool) else hex(r))})
    return out


def wide_vectors(seed=20261016):
    """Per-op vectors at widths > 256 (257: z3's no-overflow expansions; 512: keccak inputs
    and zero-padded equalities), expected values from the oracle's width-generic functions."""
    import pyoracle as O
    rng = random.Random(seed)
    names = {"bvadd": O.bvadd, "bvsub": O.bvsub, "bvand": lambda a, b, w: a & b,
             "bvxor": lambda a, b, w: a ^ b, "bvneg": lambda a, b, w: O.bvneg(a, w),
             "bvnot": lambda a, b, w: O.bvnot(a, w), "bvult": O.ult, "bvule": O.ule,
             "bvslt": O.slt, "bvsle": O.sle}
    out = []
    for w in (257, 300, 512):
        M = (1 << w) - 1
        pool = sorted({p & M for p in [0, 1, 2, M, M - 1, 1 << (w - 1), (1 << (w - 1)) - 1,
                                        (1 << 256) - 1, 1 << 256, (1 << 255) + 7]})
        for name, fn in names.items():
            pairs = [(a, b) for a in pool[::2] for b in pool[1::2]]
            pairs += [(rng.getrandbits(w), rng.getrandbits(w)) for _ in range(6)]
            for a, b in pairs:
                r = fn(a, b, w)
                out.append({"op": name, "w": w, "a": a, "b": b, "r": int(r)})
    return {"source": "oracle/pyoracle.py width-generic ops (tools/make_golden.py wide_vectors)",
            "vectors": out}


def main():
    os.makedirs(GOLD, exist_ok=True)
    if "--wide-only" in sys.argv:
        with open(os.path.join(GOLD, "wide.json"), "w") as f:
            json.dump(wide_vectors(), f, indent=0, sort_keys=True)
        return
    sets = {"vmtests.json": vmtests(), "vmsha3.json": vmsha3(), "eip145.json": eip145(),
            "ops.json": ops_vectors(), "wide.json": wide_vectors()}
    for fn, data in sets.items():
        with open(os.path.join(GOLD, fn), "w") as f:
            json.dump(data, f, indent=0, sort_keys=True)
        print(fn, len(data))


if __name__ == "__main__":
    main()
