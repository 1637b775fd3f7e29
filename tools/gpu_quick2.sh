# quick iteration: GPU parity tests, config-3 bench line, unit profile
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-q}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0 > $O/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-330
timeout -k 10 200 python -u tools/unitprof.py > $O/unitprof.log 2>&1 || { echo "UNITPROF FAILED"; tail -5 $O/unitprof.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/unitprof.log').read().split('amdgpu.ids: No such file or directory')[-1]); print(d['kernel_ms'], d['share'])"
