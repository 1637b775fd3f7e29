# config-3 bench per EXP-split variant library (no cpu baseline / corpus / keccak legs)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/benchvar
mkdir -p $O
for m in ${MS:-24 16 12}; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0 --lib mythril_amd/libpathfeas_exp$m.so > $O/b$m.log 2>&1 || { echo "BENCH $m FAILED"; tail -5 $O/b$m.log; exit 1; }
  echo "M=$m $(tail -1 $O/b$m.log | cut -c1-330)"
done
