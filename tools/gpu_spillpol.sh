# Spill policy sweep on config 3 ($VAR, default PF_VAR_SPILL_USES, over $POLS, default 1 2 3;
# product library): a short bench each, alternating $REPS times, then a WRITE_SIZE pass each
# (DESIGN.md §9).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/spillpol
mkdir -p $O
P="--no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0 --full-pass-dags 0 --quick-sat-queries 0"
for rep in $(seq 1 ${REPS:-2}); do
for SP in ${POLS:-1 2 3}; do
  env "${VAR:-PF_VAR_SPILL_USES}=$SP" timeout -k 10 200 python -u bench.py --steps ${STEPS:-5} --warmup 2 $P > $O/b_${SP}_$rep.log 2>&1 || { echo "bench $SP failed"; exit 1; }
  python -c "import json; d=json.loads(open('$O/b_${SP}_$rep.log').read().strip().splitlines()[-1]); print('pol $SP', round(d['value']/1e9,4), round(d['roofline']['kernel_ms_avg'],3))"
done
done
for SP in ${POLS:-1 2 3}; do
  env "${VAR:-PF_VAR_SPILL_USES}=$SP" timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$SP -o run -- python bench.py --steps 2 --warmup 1 $P > $O/w_$SP.log 2>&1 || { echo "pmc $SP failed"; exit 1; }
done
echo SWEEP-DONE
