# Round-end profile evidence at HEAD in one call: PMC passes (tools/gpu_profile.sh: kernel
# trace, FETCH_SIZE, WRITE_SIZE, SQ mix, clock), the SQ stall pass + unit profile
# (tools/gpu_stalls.sh; libpathfeas_prof.so built on the CPU beforehand).
cd $GRAFT_REPO_ROOT
TAG=${1:-r02d}
bash tools/gpu_profile.sh $TAG && bash tools/gpu_stalls.sh $TAG
