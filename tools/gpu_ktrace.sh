# Kernel trace of a short bench (which search kernels ran, their average duration).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0 > gpurun_out/kt/bench.log 2>&1 || { echo "trace failed"; exit 1; }
find gpurun_out/kt -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
