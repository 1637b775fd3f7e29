# PMC pass: instruction-cache behaviour of pf_check_kernel on the config-3 bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/icache
mkdir -p $O
B="python bench.py --steps 1 --warmup 0 --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0 ${BENCH_ARGS:-}"
timeout -s KILL 200 rocprofv3 --pmc ${PMC:-SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES} --output-format csv -d $O/p1 -o run -- $B > $O/p1.log 2>&1 || { echo "p1 failed"; tail -5 $O/p1.log; exit 1; }
python - <<'PY'
import csv, collections
agg = collections.defaultdict(float)
for r in csv.DictReader(open("gpurun_out/icache/p1/run_counter_collection.csv")):
    if "pf_check_kernel" in r["Kernel_Name"]:
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, "%.4g" % v)
PY
