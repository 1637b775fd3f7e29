# PMC pass: scalar data cache (instruction-stream and constant fetches) of pf_check_kernel,
# one pass per library in $LIBS
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/kcache
mkdir -p $O
i=0
for L in $LIBS; do
  i=$((i+1))
  B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0 --lib $L"
  timeout -s KILL 200 rocprofv3 --pmc ${PMC:-SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM} --output-format csv -d $O/p$i -o run -- $B > $O/p$i.log 2>&1 || { echo "p$i failed"; tail -5 $O/p$i.log; exit 1; }
  python - $i $L <<'PY'
import csv, collections, sys
agg = collections.defaultdict(float)
for r in csv.DictReader(open(f"gpurun_out/kcache/p{sys.argv[1]}/run_counter_collection.csv")):
    if r["Kernel_Name"].startswith("pf_check_kernel"):
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[2], " ".join(f"{k}={v:.4g}" for k, v in sorted(agg.items())))
PY
done
