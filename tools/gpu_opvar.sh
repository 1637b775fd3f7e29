# opbench per variant library (timing experiments): OPS and MS env vars
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/opvar
mkdir -p $O
for m in ${MS:-X0}; do
  timeout -k 10 200 python -u tools/opbench.py --sets 256 --ops ${OPS:-udiv_q1,udiv_q8,xor} --lib mythril_amd/libpathfeas_exp$m.so > $O/op$m.log 2>&1 || { echo "OPBENCH $m FAILED"; tail -5 $O/op$m.log; exit 1; }
  grep -v "^{" $O/op$m.log | grep -v amdgpu.ids | sed "s/^/$m /" | cut -c1-160
done
