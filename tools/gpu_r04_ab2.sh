# A/B timing (tools/gpu_round_ab.sh, NOTESTS) then WRITE_SIZE passes (tools/gpu_r04_wsize.sh)
cd $GRAFT_REPO_ROOT
TAG=${1:-r04e}
NOTESTS=1 NOBENCH=1 bash tools/gpu_round_ab.sh $TAG ${AB:-} || exit 1
bash tools/gpu_r04_wsize.sh $TAG ${WS:-} || exit 1
