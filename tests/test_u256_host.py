"""Host build of the kernel's 256-bit arithmetic (csrc/u256.h via tools/u256_host_check.cpp)
against Python big ints: udivrem256 on every path (zero / short / one-digit / general, and
the general path alone), mul256, sqr256, exp256 and the 2-adic EXP split, with adversarial
a = b*q + r divisions whose quotient estimates land on integer boundaries (the biased
estimates' add-back).  Each host case is a one-lane wave, so every wave-uniform fast path
is taken exactly when its own lane qualifies; mixed waves are the GPU parity tests' job
(tests/test_gpu_parity.py).  CPU only."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FUZZ = os.path.join(ROOT, "tools", "u256_fuzz.py")
CLANG = "/opt/rocm/llvm/bin/clang++"


@pytest.mark.skipif(not os.path.exists(CLANG), reason="no host clang++")
@pytest.mark.parametrize("flags", ["", "-DPF_DIV_FORCE_GENERAL"])
def test_u256_host_fuzz(flags, tmp_path):
    env = dict(os.environ, U256_FLAGS=flags, TMPDIR=str(tmp_path))
    r = subprocess.run([sys.executable, FUZZ, "4000"], capture_output=True, text=True,
                       env=env, cwd=str(tmp_path), timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert " 0 bad" in r.stdout
