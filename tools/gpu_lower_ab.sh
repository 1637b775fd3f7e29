# Native lowering A/B on the GPU box's host cores: tools/lower_bench.py per libpflower build
# (build_var/libpflower_<v>.so; "base" = the product library), alternated.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2 3; do
for v in "$@"; do
  if [ "$v" = base ]; then L=mythril_amd/libpflower.so; else L=build_var/libpflower_$v.so; fi
  PF_LOWER_SO=$L timeout -k 10 300 python tools/lower_bench.py $v || { echo "lower bench $v failed"; exit 1; }
done
done
echo LOWER-AB-DONE
