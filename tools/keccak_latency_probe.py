"""GPU box: latency of one pf_keccak256_batch call (pooled block, pinned staging, one launch)
for n 64-byte preimages, against a host Keccak-f[1600] per message (hashlib's sha3_256: the
same permutation as eth_hash's keccak, only the padding byte differs).  Sets
concretize.GPU_MIN (the batch size from which the concretisation hashes on the GPU)."""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import numpy as np  # noqa: E402

from mythril_amd.engine import get_engine  # noqa: E402

eng = get_engine()
out = []
for n in (1, 2, 4, 8, 16, 32, 64, 128, 256, 1024):
    msgs = [os.urandom(64) for _ in range(n)]
    eng.keccak256(msgs)
    ts = []
    for _ in range(30):
        t0 = time.perf_counter()
        eng.keccak256(msgs)
        ts.append(1e6 * (time.perf_counter() - t0))
    th = []
    for _ in range(30):
        t0 = time.perf_counter()
        for m in msgs:
            hashlib.sha3_256(m).digest()
        th.append(1e6 * (time.perf_counter() - t0))
    out.append({"n": n, "gpu_us_median": float(np.median(ts)), "host_us_median": float(np.median(th))})
print(json.dumps(out))
