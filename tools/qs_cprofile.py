"""cProfile of the bench's mixed-cache quick-sat workload (tests/model_cache_workload.py)
on the GPU box: where the GPU-resident ModelCache's per-query time goes.  Tool.

usage: python tools/qs_cprofile.py [top]"""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]

import model_cache_workload as W  # noqa: E402

top = int(sys.argv[1]) if len(sys.argv) > 1 else 30
pr = cProfile.Profile()
pr.enable()
r = W.quick_sat_profile(n_models=100, n_scenarios=16, n_queries=121)
pr.disable()
print({k: r[k] for k in ("reference_loop_ms", "gpu_model_cache_ms", "slowest_query", "verdicts")})
pstats.Stats(pr).sort_stats("tottime").print_stats(top)
