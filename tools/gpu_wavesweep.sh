# Waves-per-CU sweep of the full-sweep search (PF_WAVES_PER_CU overrides the geometry).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ws
for W in ${@:-256 512 768 1024}; do
  PF_WAVES_PER_CU=$W timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0 --full-pass-dags 0 --quick-sat-queries 0 > gpurun_out/ws/$W.log 2>&1 || { echo "W=$W failed"; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ws/$W.log').read().strip().splitlines()[-1]); print('$W', round(d['value']/1e9,4), 'Gevals/s', round(d['roofline']['kernel_ms_avg'],3), 'ms frac', round(d['roofline']['frac'],4))"
done
