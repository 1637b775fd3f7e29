# Round check on the GPU box: parity suite, smoke, one bench line (each step time-limited,
# chained with && so a failing step stops the call).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --cpu-sample-s 10 > gpurun_out/bench_$TAG.log 2>&1
RC=$?
echo "CHAIN EXIT $RC"
tail -3 gpurun_out/gpu_tests_$TAG.log; tail -2 gpurun_out/smoke_$TAG.log; tail -c 3000 gpurun_out/bench_$TAG.log
exit $RC
