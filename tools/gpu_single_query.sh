# The bench's discharge leg (corpus batch, hints-off, live order, single-query sample) alone,
# once per environment setting ("base" = defaults), each its own process.
# usage: bash tools/gpu_single_query.sh TAG base ENV=VALUE lib:NAME ...  (lib: build_var/lib_NAME.so)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-sq}; shift
O=gpurun_out/$TAG
mkdir -p $O
B="python -u bench.py --steps 1 --warmup 0 --sets 64 --budget 64 --keccak-log2 0 --full-pass-dags 0 --quick-sat-queries 0 --no-cpu-baseline"
i=0
for rep in 1 2; do
for v in "$@"; do
  i=$((i+1))
  E=""; L=""
  if [ "${v#lib:}" != "$v" ]; then L="--lib build_var/lib_${v#lib:}.so"; elif [ "$v" != base ]; then E="$v"; fi
  timeout -k 10 300 env $E $B $L > $O/sq$i.log 2>&1 || { echo "variant $v failed"; tail -5 $O/sq$i.log; exit 1; }
  python -c "
import json; d=json.loads(open('$O/sq$i.log').read().strip().splitlines()[-1])['discharge']
s=d['single_query_ms']; print('$v', {k: round(s[k],3) for k in ('median','mean','p95','max')}, s['phase_mean_ms'], 'qps', round(d['queries_per_s']), 'pct', round(d['pct_discharged_builder_corpus'],1))"
done
done
echo SQ-DONE
