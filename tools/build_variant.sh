#!/bin/bash
# Build tools/bin/lib<NAME>.so: the tree's objects (flyimg_amd/build, run make
# first) with one source replaced by SRC compiled with FLAGS.  For A/B runs
# through FI_LIB_PATH (tools/gpu_abl.sh).  SRC may be a file outside csrc
# (e.g. a `git show HEAD:...` copy); it is compiled with csrc on the include path.
#   tools/build_variant.sh base /tmp/head/fi_smartcrop.hip ""
#   tools/build_variant.sh pair1 flyimg_amd/csrc/fi_smartcrop.hip "-DFI_FZ_PAIR=1"
set -eu
cd "$(dirname "$0")/.."
NAME=$1 SRC=$2 FLAGS=${3:-}
ROCM=${ROCM:-/opt/rocm}
B=flyimg_amd/build
obj=$(basename "$SRC").o
[ -f "$B/$obj" ] || { echo "no $B/$obj to replace"; exit 1; }
tmp=$(mktemp -d)
$ROCM/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Iflyimg_amd/csrc -Iinclude $FLAGS -c "$SRC" -o "$tmp/$obj"
objs=""
for o in $B/*.o; do
  if [ "$(basename $o)" = "$obj" ]; then objs="$objs $tmp/$obj"; else objs="$objs $o"; fi
done
mkdir -p tools/bin
$ROCM/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/bin/lib$NAME.so $objs -L$ROCM/lib -lrccl -Wl,-rpath,$ROCM/lib
rm -rf "$tmp"
echo tools/bin/lib$NAME.so
