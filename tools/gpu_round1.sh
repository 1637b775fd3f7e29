cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests_r1c.log 2>&1
echo "TESTS EXIT $?" >> gpurun_out/gpu_tests_r1c.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r1c.log 2>&1 && \
timeout -k 10 300 python bench.py --sets 256 --steps 2 --warmup 1 --cpu-sample-s 5 > gpurun_out/bench_small_r1c.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --cpu-sample-s 10 > gpurun_out/bench_r1c.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1c -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof_r1c.log 2>&1
echo "CHAIN EXIT $?"
tail -3 gpurun_out/gpu_tests_r1c.log; cat gpurun_out/smoke_r1c.log | tail -2; cat gpurun_out/bench_small_r1c.log | tail -3; cat gpurun_out/bench_r1c.log | tail -2
