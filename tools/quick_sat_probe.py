"""GPU box: bench.py's quick-sat leg alone (100 cached models; witness / mixed caches; the
stand-in funnel), one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import bench  # noqa: E402

args = bench.parse(sys.argv[1:])
print(json.dumps(bench.quick_sat_leg(args)), flush=True)
