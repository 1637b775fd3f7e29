# The bench's quick_sat leg alone (a tiny config-3 step in front), once per environment
# setting given as arguments ("base" = defaults), each its own process.
# usage: bash tools/gpu_quicksat.sh TAG base PF_QS_HOST_PAIRS=0 PF_QS_MEMO=0 ...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-qs}; shift
O=gpurun_out/$TAG
mkdir -p $O
B="python -u bench.py --steps 1 --warmup 0 --sets 64 --budget 64 --keccak-log2 0 --full-pass-dags 0 --corpus-scenarios 0 --no-cpu-baseline --quick-sat-queries ${QSQ:-121}"
i=0
for v in "$@"; do
  i=$((i+1))
  E=""; [ "$v" != base ] && E="$v"
  timeout -k 10 300 env $E $B > $O/qs$i.log 2>&1 || { echo "variant $v failed"; tail -5 $O/qs$i.log; exit 1; }
  python -c "
import json; d=json.loads(open('$O/qs$i.log').read().strip().splitlines()[-1])['quick_sat']
for k in ('witness_cache','mixed_cache'):
    q=d[k]; print('$v', k, 'ref', q['reference_loop_ms'], 'gpu', q['gpu_model_cache_ms'], 'agree', q['choices_agree'], '/', q['queries'], 'calls', q['engine_calls'], q.get('verdicts'), q['phase_ms_per_query'])
f=d['funnel']; print('$v funnel', f['funnel_query_ms'], f['phase_mean_ms'])"
done
echo QS-DONE
