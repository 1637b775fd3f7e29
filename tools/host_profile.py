"""Where the native lowering's time goes on single queries (DESIGN §4 host cost): the
bench's 96-query single-query sample lowered with hints (native_terms.lower_many, one thread)
under tools/libsampler.so (SIGPROF sampling of the instruction pointer), samples mapped to
libpflower.so symbols with nm.  CPU only: concrete keccak values come from the Python oracle,
no engine is used.  Tool (tools/, not product).

usage: python tools/host_profile.py [reps] [top]
"""
import bisect
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import pyoracle as O  # noqa: E402

from mythril_amd import corpus, keccak_manager as KM  # noqa: E402
from mythril_amd.smt import gpu_check, native_terms, symbol_factory  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    so = os.path.join(ROOT, "tools", "libsampler.so")
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(ROOT, "tools", "sampler.c")],
                   check=True)
    S = ctypes.CDLL(so)
    S.sampler_stop.restype = ctypes.c_size_t
    KM.KeccakFunctionManager.find_concrete_keccak = staticmethod(lambda data: symbol_factory.BitVecVal(
        int.from_bytes(O.keccak256(data.value.to_bytes(data.size() // 8, "big")), "big"), 256))
    c = corpus.build(48, 2, seed=2024)
    sample = [q for q in c.queries if q.label == "sat"][:96]
    reg = c.kfm.registry
    jobs = []
    for q in sample:
        bks = native_terms.buckets(list(q.constraints))
        jobs.append(([(b, None) for b in bks], [gpu_check._set_seed(b) for b in bks]))
    for j, seeds in jobs:  # warm
        native_terms.lower_many(j, reg, True, seeds, 1)
    S.sampler_start(100)
    for _ in range(reps):
        for j, seeds in jobs:
            native_terms.lower_many(j, reg, True, seeds, 1)
    buf = (ctypes.c_uint64 * (1 << 20))()
    n = S.sampler_stop(buf, 1 << 20)
    ips = np.frombuffer(buf, dtype=np.uint64, count=n)
    # map: the loaded libpflower.so's base from /proc/self/maps, symbols from nm
    lib = os.path.join(ROOT, "mythril_amd", "libpflower.so")
    base = None
    for line in open("/proc/self/maps"):
        if line.rstrip().endswith(lib) and " 00000000 " in line:
            base = int(line.split("-")[0], 16)
            break
    syms = []
    for line in subprocess.run(["nm", "-C", "--defined-only", "-n", lib], capture_output=True,
                               text=True).stdout.splitlines():
        parts = line.split(" ", 2)
        if len(parts) == 3 and parts[1].lower() in ("t", "w"):
            syms.append((int(parts[0], 16), parts[2]))
    addrs = [a for a, _ in syms]
    maps = []
    for line in open("/proc/self/maps"):
        f = line.split()
        if len(f) >= 6 and "x" in f[1]:
            lo, hi = (int(x, 16) for x in f[0].split("-"))
            maps.append((lo, hi, os.path.basename(f[5])))
    where = {}
    for ip in ips.tolist():
        name = next((m[2] for m in maps if m[0] <= ip < m[1]), "?")
        where[name] = where.get(name, 0) + 1
    print("samples by mapping:", sorted(where.items(), key=lambda kv: -kv[1])[:8])
    # libc: which functions (allocation churn shows up here)
    libc = next((line.split()[5] for line in open("/proc/self/maps")
                 if line.split()[-1].endswith("libc.so.6") and " 00000000 " in line), None)
    if libc:
        lbase = next(int(line.split("-")[0], 16) for line in open("/proc/self/maps")
                     if line.split()[-1] == libc and " 00000000 " in line)
        ls = []
        for line in subprocess.run(["nm", "-D", "--defined-only", "-n", libc], capture_output=True,
                                   text=True).stdout.splitlines():
            parts = line.split(" ", 2)
            if len(parts) == 3 and parts[1].lower() in ("t", "w", "i"):
                ls.append((int(parts[0], 16), parts[2]))
        la = [a for a, _ in ls]
        lc = {}
        for ip in ips.tolist():
            off = ip - lbase
            i = bisect.bisect_right(la, off) - 1
            if 0 <= i and 0 <= off - la[i] < 1 << 16:
                lc[ls[i][1]] = lc.get(ls[i][1], 0) + 1
        print("libc:", sorted(lc.items(), key=lambda kv: -kv[1])[:10])
    counts = {}
    outside = 0
    for ip in ips.tolist():
        off = ip - base if base is not None else -1
        i = bisect.bisect_right(addrs, off) - 1
        if off < 0 or i < 0 or off - addrs[i] > 1 << 16:
            outside += 1
            continue
        counts[syms[i][1]] = counts.get(syms[i][1], 0) + 1
    print(f"{n} samples, {outside} outside libpflower.so")
    for name, k in sorted(counts.items(), key=lambda kv: -kv[1])[:top]:
        print(f"{100.0 * k / max(n, 1):6.2f}%  {name[:150]}")


if __name__ == "__main__":
    main()
