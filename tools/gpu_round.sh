# One GPU call: gpu parity tests, smoke, bench (default config), kernel-trace profile.
# usage: bash tools/gpu_round.sh TAG
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r01}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --corpus-scenarios 0 ${BENCH_ARGS:-} > $O/trace.log 2>&1 || { echo "TRACE FAILED"; tail -20 $O/trace.log; exit 1; }
echo ROUND-DONE
