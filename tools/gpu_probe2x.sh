# Doubling probes (pf_eval.hip PF_PROBE_2X_*): the product library and each probe build, one
# short config-3 bench each (no full pass, no host legs), A/B order repeated against drift.
# usage: bash tools/gpu_probe2x.sh TAG variant1 variant2 ...   (build_var/lib_<v>.so)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-p2x}; shift
O=gpurun_out/$TAG
mkdir -p $O
B="python -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0 --full-pass-dags 0 --quick-sat-queries 0"
i=0
for rep in $(seq ${REPS:-2}); do
for v in base "$@"; do
  i=$((i+1))
  if [ "$v" = base ]; then L=""; else L="--lib build_var/lib_$v.so"; fi
  timeout -k 10 200 $B $L > $O/ab$i.log 2>&1 || { echo "variant $v failed"; tail -5 $O/ab$i.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/ab$i.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value']/1e9,4), 'Gevals/s', round(r['kernel_ms_avg'],3), 'ms frac', round(r['frac'],4))"
done
done
echo AB-DONE
