# quick GPU check: parity tests (mul/exp focused first), micro-benchmark, opbench subset
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-quick}
OPS=${2:-add,mul,exp,udiv,urem}
timeout -k 10 120 ./tools/mulbench > gpurun_out/mulbench_$TAG.log 2>&1; echo "MULBENCH EXIT $?"; cat gpurun_out/mulbench_$TAG.log
timeout -k 10 300 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -3 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/opbench.py --sets 256 --ops $OPS > gpurun_out/opbench_$TAG.log 2>&1
rc=$?; grep -v "^{" gpurun_out/opbench_$TAG.log | grep -v amdgpu.ids | cut -c1-200
exit $rc
