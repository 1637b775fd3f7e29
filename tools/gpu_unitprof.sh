cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/unitprof.py --sets 1024 > gpurun_out/unitprof.json 2> gpurun_out/unitprof.err && \
timeout -k 10 300 python -u tools/opbench.py --sets 256 --ops add,xor,var,mul,udiv,ult_ite,concat8 > gpurun_out/opbench.log 2>&1
RC=$?
cat gpurun_out/unitprof.json | head -20; tail -8 gpurun_out/opbench.log | cut -c1-200
exit $RC
