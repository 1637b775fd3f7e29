cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gq_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0 > gpurun_out/gq_bench.log 2>&1
RC=$?
tail -3 gpurun_out/gq_tests.log
python -c "import json; d=json.loads(open('gpurun_out/gq_bench.log').read().strip().splitlines()[-1]); print(d['value']/1e9, 'Gevals/s', d['roofline']['kernel_ms_avg'], 'ms frac', d['roofline']['frac'], 'hw', d['roofline'].get('hw'))"
exit $RC
