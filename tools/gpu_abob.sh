# A/B of two library builds: GPU parity tests on the product library, config-3 bench and
# the opbench chains (dependent vs interleaved) for each of $LIBS.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/abob_${1:-x}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
i=0
for L in $LIBS; do
  i=$((i+1))
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0 --lib $L > $O/b$i.log 2>&1 || { echo "BENCH $L FAILED"; tail -5 $O/b$i.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b$i.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$L', round(d['value']/1e9,4), 'Gevals/s', round(r['kernel_ms_avg'],3), 'ms frac', round(r['frac'],4))"
  timeout -k 10 200 python -u tools/opbench.py --sets 2048 --ops ${OPS:-add1,add4,mul1,mul4} --lib $L > $O/o$i.log 2>&1 || { echo "OPBENCH $L FAILED"; tail -5 $O/o$i.log; exit 1; }
  grep -E "^[a-z0-9_]+ \{" $O/o$i.log | cut -c1-48
done
