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
