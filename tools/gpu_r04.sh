# Round-4 GPU call: parity suite + smoke + default bench on the product library, then the
# A/B variants given as arguments (tools/gpu_round_ab.sh), then tools/movbench at 4 and 8
# waves per SIMD (latency-limited issue rates, incl. v_bitop3_b32 / v_alignbit_b32).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r04}; shift
bash tools/gpu_round_ab.sh $TAG "$@" || exit 1
O=gpurun_out/$TAG
if [ -x tools/movbench ]; then
  for w in 4 8; do timeout -k 10 120 ./tools/movbench $w >> $O/movbench.log 2>&1 || { echo "movbench failed"; exit 1; }; done
  echo MOVBENCH-DONE
fi
# Keccak variants (KECCAK="kp6 kp8"): one process per library, the product first and last
if [ -n "$KECCAK" ]; then
  for v in base $KECCAK base; do
    if [ "$v" = base ]; then L=""; else L="--lib build_var/lib_$v.so"; fi
    timeout -k 10 120 python -u tools/keccak_ab.py $L >> $O/keccak_ab.log 2>&1 || { echo "keccak $v failed"; tail -5 $O/keccak_ab.log; exit 1; }
  done
  cat $O/keccak_ab.log | grep ms_median
fi
