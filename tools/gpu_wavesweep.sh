# Launch-geometry sweep: config-3 full sweep at several waves-per-CU targets.
# usage: bash tools/gpu_wavesweep.sh TAG
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-wsweep}
mkdir -p $O
for w in ${WLIST:-64 128 256 512 1024}; do
  PF_WAVES_PER_CU=$w timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0 > $O/w$w.log 2>&1 || { echo "BENCH w=$w FAILED"; tail -20 $O/w$w.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/w$w.log').read().strip().splitlines()[-1]); print($w, d['value'], d['roofline']['kernel_ms_avg'], d['early_exit']['kernel_ms'])"
done
echo SWEEP-DONE
