# GPU check after an EXP / interpreter change: parity tests, opbench (exp, mul), bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-exp}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -u tools/opbench.py --sets 256 --ops ${OPS:-exp,mul,udiv,add} > $O/opbench.log 2>&1 || { echo "OPBENCH FAILED"; tail -20 $O/opbench.log; exit 1; }
grep -v "^{" $O/opbench.log | grep -v amdgpu.ids | cut -c1-200
timeout -k 10 400 python -u bench.py --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0 > $O/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-700
echo DONE
