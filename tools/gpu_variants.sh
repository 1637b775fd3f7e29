# Time alternative builds of libpathfeas.so on the default config-3 bench (no parity claim:
# a variant may change the generator contract; only kernel time is compared).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/var
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0 --full-pass-dags 0 --quick-sat-queries 0"
for v in base "$@"; do
  if [ "$v" = base ]; then L=""; else L="--lib build_var/lib_$v.so"; fi
  timeout -k 10 300 $B $L > gpurun_out/var/$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/var/$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e9,4), 'Gevals/s', round(d['roofline']['kernel_ms_avg'],3), 'ms', 'frac', round(d['roofline']['frac'],4))"
done
