# Round-4 profile call: GPU parity suite, then tools/gpu_profile.sh (kernel trace + PMC passes)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r04d}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/$TAG/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$TAG/gpu_tests.log
bash tools/gpu_profile.sh $TAG || exit 1
