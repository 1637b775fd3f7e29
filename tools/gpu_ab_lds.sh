cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
LIBS="build_var/lib_nolds.so mythril_amd/libpathfeas.so" REPS="1 2" bash tools/gpu_ab.sh lds || exit 1
O=gpurun_out/ab_lds
P="--steps 2 --warmup 1 --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0 --full-pass-dags 0 --quick-sat-queries 0"
for L in build_var/lib_nolds.so mythril_amd/libpathfeas.so; do
  n=$(basename $L .so)
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$n -o run -- python bench.py $P --lib $L > $O/w_$n.log 2>&1 || { echo "pmc $n failed"; exit 1; }
done
echo AB-DONE
