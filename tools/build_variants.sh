# Build timing variants of libpathfeas.so into build_var/lib_<name>.so: each argument is
# name=FLAGS (e.g. nolaser=-DPF_DIAG_NO_LASER_ARMS).  Host-side (hipcc cross-compiles).
cd "$(dirname "$0")/.."
mkdir -p build_var
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-value \
    -mllvm -structurizecfg-skip-uniform-regions=true $flags \
    -o build_var/lib_$name.so mythril_amd/csrc/pathfeas.hip &
done
wait
ls -la build_var
