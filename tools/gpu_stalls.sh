# Wave-time breakdown of pf_check_kernel (one PMC pass, 8 SQ counters) + per-unit time shares
# (tools/unitprof.py, profiling build libpathfeas_prof.so built on the CPU beforehand).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r02}
OUT=gpurun_out/stalls_$TAG
mkdir -p $OUT
P="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/st -o run -- $P > $OUT/st.log 2>&1 || { echo "stall pass failed"; exit 1; }
timeout -k 10 300 python tools/unitprof.py > $OUT/unitprof.json 2> $OUT/unitprof.err || { echo "unitprof failed"; exit 1; }
python tools/stall_summary.py $OUT/st > $OUT/st.md 2>&1 || true
cat $OUT/st.md; cat $OUT/unitprof.json
