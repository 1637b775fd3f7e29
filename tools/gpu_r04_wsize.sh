# WRITE_SIZE per launch of pf_check_kernel for libraries / spill policies (one rocprofv3 --pmc
# pass each).  usage: bash tools/gpu_r04_wsize.sh TAG v1 v2 ... ("base", a build_var name, or
# "sp:N" = product library with PF_VAR_SPILL_USES=N)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-x}; shift
O=gpurun_out/$TAG/wsize
mkdir -p $O
P="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --corpus-scenarios 0 --keccak-log2 0"
for v in "$@"; do
  L=""; SP=1
  if [ "${v#sp:}" != "$v" ]; then SP="${v#sp:}"; elif [ "$v" != base ]; then L="--lib build_var/lib_$v.so"; fi
  PF_VAR_SPILL_USES=$SP timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$v -o run -- $P $L > $O/$v.log 2>&1 || { echo "wsize $v failed"; exit 1; }
done
echo WSIZE-DONE
