# Occupancy experiment (diagnostic, no parity claim): kernel builds with smaller register
# banks / more waves per SIMD, each paired with a lowering build of matching PF_NW.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/occ
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0"
run() {  # name lib lower_so
  PF_LOWER_SO=$3 timeout -k 10 300 $B $2 > gpurun_out/occ/$1.log 2>&1 || { echo "variant $1 failed"; tail -5 gpurun_out/occ/$1.log; return 1; }
  python -c "import json; d=json.loads(open('gpurun_out/occ/$1.log').read().strip().splitlines()[-1]); print('$1', round(d['value']/1e9,4), 'Gevals/s', round(d['roofline']['kernel_ms_avg'],3), 'ms frac', round(d['roofline']['frac'],4))"
}
run base "" "" && \
run b8w2 "--lib build_var/lib_b8w2.so" build_var/libpflower_nw7.so && \
run b8w3 "--lib build_var/lib_b8w3.so" build_var/libpflower_nw7.so && \
run b8w4 "--lib build_var/lib_b8w4.so" build_var/libpflower_nw7.so
