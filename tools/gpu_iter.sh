# one GPU iteration: parity tests, per-op bench, headline bench (each step bounded)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-iter}
timeout -k 10 300 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -3 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/opbench.py --sets 256 > gpurun_out/opbench_$TAG.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --cpu-sample-s 10 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "BENCH EXIT $rc"
grep -v "^{" gpurun_out/opbench_$TAG.log | grep -v amdgpu.ids; tail -1 gpurun_out/bench_$TAG.log
exit $rc
