#!/usr/bin/env python3
"""Config-4 Keccak timing of one libpathfeas.so build (A/B of kernel variants, one process per
library): 2^k 64-byte preimages resident in HBM, pf_keccak256_fixed_dev HIP-event time per
launch, the VALU issue fraction at 4,340 instructions per wave, and a digest check of a
sample against the C oracle."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--log2", type=int, default=24)
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    import torch

    from mythril_amd import _lib
    if a.lib:
        _lib.load_library(a.lib)
    _lib.init(0)
    n = 1 << a.log2
    g = torch.Generator(device="cuda").manual_seed(7)
    data = torch.randint(0, 256, (n * 64,), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    L = _lib.lib()
    ms = ctypes.c_float(0)
    st = torch.cuda.current_stream().cuda_stream
    t = []
    for k in range(a.reps + 2):
        _lib.check(L.pf_keccak256_fixed_dev(data.data_ptr(), 64, n, out.data_ptr(), ctypes.byref(ms), st), "keccak")
        if k >= 2:
            t.append(ms.value)
    torch.cuda.synchronize()
    import coracle_py
    h = data.cpu().numpy().reshape(n, 64)
    o = out.cpu().numpy().reshape(n, 32)
    idx = np.array(sorted(set(np.random.default_rng(1).choice(n, 4096, replace=False).tolist() + [0, n - 1])))
    want = coracle_py.keccak256_fixed(h[idx], 64, len(idx))
    bad = int((want != o[idx]).any(axis=1).sum())
    m = float(np.median(t))
    print(json.dumps({"lib": a.lib or "product", "ms_median": m, "ms_min": float(min(t)),
                      "hashes_per_s": n / (m / 1e3),
                      "valu_issue_frac": (n / 64) * 4340 * 2 / (1024 * 2.4e9 * m / 1e3),
                      "digest_mismatches": int(bad), "checked": len(idx)}))


if __name__ == "__main__":
    main()
