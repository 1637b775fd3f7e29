# EXP split variants: parity (product build), then opbench exp per variant library.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/expvar
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "exp" > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for m in ${MS:-30 24 20 16 12 8}; do
  timeout -k 10 120 python -u tools/opbench.py --sets 256 --ops exp --lib mythril_amd/libpathfeas_exp$m.so > $O/op$m.log 2>&1 || { echo "OPBENCH $m FAILED"; tail -5 $O/op$m.log; exit 1; }
  echo "M=$m $(grep '^exp' $O/op$m.log | cut -c1-200)"
done
