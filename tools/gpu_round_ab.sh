# One GPU call: parity tests + smoke + default bench on the product library, then a short
# config-3 bench per variant library (build_var/lib_<name>.so, tools/build_variants.sh) with
# the product library between them (A/B/A order against box drift).
# usage: bash tools/gpu_round_ab.sh TAG variant1 variant2 ...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-x}; shift
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "$NOTESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $O/bench.log; exit 1; }
  tail -1 $O/bench.log | cut -c1-400
fi
B="python -u bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0"
i=0
for rep in 1 2; do
for v in base "$@"; do
  i=$((i+1))
  # a variant "env:NAME=VALUE" runs the product library with that environment variable
  # (host-side policies, e.g. the lowering's PF_VAR_SPILL_USES); any other name is a library
  E=""
  if [ "$v" = base ]; then L=""; elif [ "${v#env:}" != "$v" ]; then L=""; E="${v#env:}"; else L="--lib build_var/lib_$v.so"; fi
  timeout -k 10 200 env $E $B $L > $O/ab$i.log 2>&1 || { echo "variant $v failed"; tail -5 $O/ab$i.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/ab$i.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value']/1e9,4), 'Gevals/s', round(r['kernel_ms_avg'],3), 'ms frac', round(r['frac'],4), 'early', round(d['early_exit']['unplanted']['kernel_ms'],3), round(d['early_exit']['planted']['kernel_ms'],3))"
done
done
echo AB-DONE
# parity of variant builds (PARITY="v1 v2"): the box's scratch copy of the product library is
# replaced by the variant, then the GPU parity files run against it
cp mythril_amd/libpathfeas.so $O/libpathfeas_product.so
for v in ${PARITY:-}; do
  cp build_var/lib_$v.so mythril_amd/libpathfeas.so
  timeout -k 10 300 python -u -m pytest ${PARITY_TESTS:-tests/test_gpu_parity.py tests/test_gpu_parity_scale.py tests/test_wide.py tests/test_power.py} -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/parity_$v.log 2>&1 || { echo "PARITY $v FAILED"; tail -30 $O/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $O/parity_$v.log)"
done
cp $O/libpathfeas_product.so mythril_amd/libpathfeas.so; rm -f $O/libpathfeas_product.so
