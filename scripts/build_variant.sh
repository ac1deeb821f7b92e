#!/bin/bash
# Build a variant of libgpqhe.so with extra compile flags for same-box A/B runs:
#   bash scripts/build_variant.sh NAME "-DFOO=1 -DBAR"
#   SRC=/path/to/other/csrc bash scripts/build_variant.sh NAME   (another tree)
# -> hectr_amd/lib_var/NAME/libgpqhe.so (bench / tests pick it with
# GPQHE_LIB=hectr_amd/lib_var/NAME/libgpqhe.so).  Delete lib_var/ after the
# A/B: it travels to the GPU box with every gpurun call.
set -e
cd "$(dirname "$0")/.."
NAME=$1
EXTRA=$2
SRC=${SRC:-hectr_amd/csrc}
B=/tmp/gpqhe_var_$NAME
mkdir -p $B hectr_amd/lib_var/$NAME
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result $EXTRA"
pids=()
for f in kernels.hip ks_split.hip cols_f64.hip cols_mixed.hip gemv_win.hip host_math.cpp api.cpp; do
  /opt/rocm/bin/hipcc $FLAGS -x hip -c $SRC/$f -o $B/$f.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc $FLAGS -shared -Wl,-Bsymbolic -Wl,--no-undefined $B/*.o -o $B/libgpqhe.so
mv -f $B/libgpqhe.so hectr_amd/lib_var/$NAME/libgpqhe.so
echo "built hectr_amd/lib_var/$NAME/libgpqhe.so"
