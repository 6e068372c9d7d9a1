# tools/_old/libdc_core.so from a commit's sources (default HEAD), for tools/gpu_ab_old.sh
#   bash tools/build_old.sh [REV]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:-HEAD}
T=$(mktemp -d)
mkdir -p $T/include $T/csrc $R/tools/_old
for f in $(git -C $R ls-tree --name-only $REV include/); do git -C $R show $REV:$f > $T/include/$(basename $f); done
for f in $(git -C $R ls-tree --name-only $REV data_compression_amd/csrc/); do git -C $R show $REV:$f > $T/csrc/$(basename $f); done
for s in dc_core dc_host; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I$T/include -I$T/csrc -c $T/csrc/$s.hip -o $T/$s.o
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/_old/libdc_core.so $T/dc_core.o $T/dc_host.o
rm -rf $T
echo "tools/_old/libdc_core.so from $(git -C $R rev-parse --short $REV)"
