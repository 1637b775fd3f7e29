# Early-exit search A/B: GPU parity tests on the product library, then the bench's early-exit
# legs (unplanted / planted kernel ms) for each library in $LIBS and each early-exit launch
# geometry in $EARLY_WPC: tokens WAVES[:CHUNK] (PF_WAVES_PER_CU_EARLY, PF_EARLY_CHUNK_GROUPS;
# "-" = the library's defaults).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/early_${1:-x}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
i=0
for L in $LIBS; do
for W in ${EARLY_WPC:--}; do
  i=$((i+1))
  unset PF_WAVES_PER_CU_EARLY PF_EARLY_CHUNK_GROUPS
  if [ "$W" != "-" ]; then
    export PF_WAVES_PER_CU_EARLY=${W%%:*}
    case "$W" in *:*) export PF_EARLY_CHUNK_GROUPS=${W##*:};; esac
  fi
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --corpus-scenarios ${CORPUS:-0} --keccak-log2 0 --lib $L > $O/b$i.log 2>&1 || { echo "BENCH $L $W FAILED"; tail -5 $O/b$i.log; exit 1; }
  python -c "import json; d=json.loads(open('$O/b$i.log').read().strip().splitlines()[-1]); e=d['early_exit']; q=d.get('discharge') or {}; print('$L', 'wpc=$W', round(d['value']/1e9,4), 'Gevals/s', 'unplanted', round(e['unplanted']['kernel_ms'],3), 'ms', e['unplanted']['sets_with_witness'], 'planted', round(e['planted']['kernel_ms'],3), 'ms', round(e['planted']['set_verdicts_per_s']), '/s', 'sq', (q.get('single_query_ms') or {}).get('median'))"
done
done
