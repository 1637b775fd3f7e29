# Round profile evidence at HEAD (each rocprofv3 pass its own run; no tracing domains with --pmc):
#  1. kernel-trace + stats of the bench (timed full sweep = pf_check_kernel, early-exit legs =
#     pf_check_early_kernel, Keccak = pf_keccak_fixed_kernel: separate rows)
#  2. PMC FETCH_SIZE, 3. PMC WRITE_SIZE (HBM traffic, separate passes: TCC slot budget)
#  4. PMC SQ instruction mix / wave cycles, 5. effective clock + VALU activity
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --corpus-scenarios 0 --full-pass-dags 0 --quick-sat-queries 0"
P="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --corpus-scenarios 0 --full-pass-dags 0 --quick-sat-queries 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $P > $OUT/fetch.log 2>&1 || { echo "fetch failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $P > $OUT/write.log 2>&1 || { echo "write failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVE_CYCLES --output-format csv -d $OUT/sq -o run -- $P > $OUT/sq.log 2>&1 || { echo "sq failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $OUT/clk -o run -- $P > $OUT/clk.log 2>&1 || { echo "clk failed"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT --output-format csv -d $OUT/f64 -o run -- $P > $OUT/f64.log 2>&1 || { echo "f64 failed"; exit 1; }
echo PROFILE-DONE
tail -1 $OUT/trace.log | cut -c1-300
# optional: WRITE_SIZE with another lowering spill policy (SPILLPOL=N -> PF_VAR_SPILL_USES=N)
if [ -n "$SPILLPOL" ]; then
  PF_VAR_SPILL_USES=$SPILLPOL timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_sp$SPILLPOL -o run -- $P > $OUT/write_sp$SPILLPOL.log 2>&1 || { echo "write_sp failed"; exit 1; }
  echo SPILLPOL-DONE
fi
