# PMC passes (each its own rocprofv3 run, no tracing domains): instruction mix and stalls
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
TAG=${1:-pmc}
OPS=${2:-add,mul,exp,urem,udiv,var}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVE_CYCLES"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_IFETCH SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc/${TAG}_op$i -o run -- python tools/opbench.py --sets 128 --ops $OPS > gpurun_out/pmc/${TAG}_op$i.log 2>&1 || { echo "op pass $i failed"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc/${TAG}_bench$i -o run -- python bench.py --sets 512 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc/${TAG}_bench$i.log 2>&1 || { echo "bench pass $i failed"; exit 1; }
done
echo PMC-DONE
find gpurun_out/pmc -name "*.csv" | head
