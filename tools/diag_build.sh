# diagnostic/ablation build of libdc_core.so into tools/<OUT>/ (pass -DDC_DIAG for s_memtime stamps)
#   bash tools/diag_build.sh [OUT=_diag] [EXTRA_FLAGS]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-_diag}; EXTRA=${2:-}
mkdir -p $R/tools/$OUT
for s in dc_core dc_host; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $EXTRA -I$R/include -I$R/data_compression_amd/csrc \
    -c $R/data_compression_amd/csrc/$s.hip -o $R/tools/$OUT/$s.o 2>/dev/null
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/$OUT/libdc_core.so $R/tools/$OUT/dc_core.o $R/tools/$OUT/dc_host.o
