#!/usr/bin/env python3
"""Fuzz tools/u256_host_check.cpp (host build of csrc/u256.h) against Python big ints:
udivrem256, mul256, sqr256, exp256, exp256_split.  Usage: python3 tools/u256_fuzz.py [n]"""
import os
import random
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
M = (1 << 256) - 1
CLANG = "/opt/rocm/llvm/bin/clang++"


def vals(rng):
    k = rng.randrange(9)
    if k == 0:
        return rng.choice([0, 1, 2, 3, 255, 256, 257, M, M - 1, 1 << 255, (1 << 255) - 1, (1 << 128),
                           (1 << 160) - 1, (1 << 84) - 1, 1 << 84, (1 << 84) + 1, (1 << 254) - 1,
                           1 << 254, (1 << 254) + 1])
    if k == 1:
        return rng.getrandbits(rng.randrange(1, 257))
    if k == 2:
        return ((1 << rng.randrange(256)) + rng.choice([-1, 0, 1])) & M
    return rng.getrandbits(256)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    exe = os.path.join(tempfile.gettempdir(), f"u256_host_check_{os.getpid()}")
    extra = os.environ.get("U256_FLAGS", "").split()
    subprocess.check_call([CLANG, "-O2", "-std=c++17", *extra, "-o", exe, os.path.join(HERE, "u256_host_check.cpp")])
    rng = random.Random(1234)
    cases = [(vals(rng), vals(rng)) for _ in range(n)]
    # adversarial divisions: a = b q + r with the remainder at the edges (r = 0, 1, b - 1,
    # b - 2) and b, q of every limb length, so quotient-digit estimates land right at an
    # integer boundary (the biased estimate's add-back path, and exact multiples)
    for _ in range(n // 2):
        b = rng.getrandbits(rng.randrange(1, 257)) | 1
        q = rng.getrandbits(rng.randrange(1, 257))
        r = rng.choice([0, 1, b - 1, b - 2, rng.randrange(b)]) % b
        a = b * q + r
        if a <= M:
            cases.append((a, b))
    inp = "".join(f"x {a:064x} {b:064x}\n" for a, b in cases)
    out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout.split("\n")
    bad = 0
    for (a, b), line in zip(cases, out):
        q, r, m, sq, ex, ex2 = (int(t, 16) for t in line.split())
        wq = M if b == 0 else a // b
        wr = a if b == 0 else a % b
        pw = pow(a, b, 1 << 256)
        want = (wq, wr, (a * b) & M, (a * a) & M, pw, pw)
        if (q, r, m, sq, ex, ex2) != want:
            bad += 1
            if bad < 5:
                print("MISMATCH", hex(a), hex(b))
    print(f"{len(cases)} cases, {bad} bad")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
