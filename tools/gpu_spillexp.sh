# The EXP-aware variable spill policy (PF_VAR_SPILL_USES_EXP, default 99) at HEAD: GPU tests,
# then config 3 A/B against the old rule (0) with WRITE_SIZE passes (tools/gpu_spillpol.sh),
# then the single-query sample under both (LASER buckets: no latency regression).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/spillexp_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/spillexp_tests.log; exit 1; }
tail -1 gpurun_out/spillexp_tests.log
VAR=PF_VAR_SPILL_USES_EXP POLS="0 99" REPS=3 STEPS=10 bash tools/gpu_spillpol.sh || exit 1
for e in 0 99 0 99; do
  echo "== PF_VAR_SPILL_USES_EXP=$e" >> gpurun_out/spillexp_sq.log
  env PF_VAR_SPILL_USES_EXP=$e timeout -k 10 200 python -u tools/single_query_probe.py 48 2 >> gpurun_out/spillexp_sq.log 2>&1 || exit 1
done
grep -E "^==|^median" gpurun_out/spillexp_sq.log
