cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1
echo "LIST EXIT $?"
timeout -k 10 500 python tools/opbench.py --sets 256 > gpurun_out/opbench_r1.log 2>&1
echo "OPBENCH EXIT $?"
tail -20 gpurun_out/opbench_r1.log
