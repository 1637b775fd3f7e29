# A/B of library builds on config 3: GPU parity tests on the product library (unless
# NOTESTS=1), then a short bench per library in $LIBS (paths relative to the repo root).
# usage: LIBS="mythril_amd/libpf_head.so mythril_amd/libpathfeas.so" bash tools/gpu_ab.sh TAG
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_${1:-x}
mkdir -p $O
if [ -z "$NOTESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
i=0
for rep in ${REPS:-1}; do
for L in $LIBS; do
  i=$((i+1))
  timeout -k 10 200 python -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0 --full-pass-dags 0 --quick-sat-queries 0 --lib $L > $O/b$i.log 2>&1 || { echo "BENCH $L FAILED"; tail -5 $O/b$i.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/b$i.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$L', round(d['value']/1e9,4), 'Gevals/s', round(r['kernel_ms_avg'],3), 'ms frac', round(r['frac'],4), 'early', round(d['early_exit']['unplanted']['kernel_ms'],3), round(d['early_exit']['planted']['kernel_ms'],3))"
done
done
