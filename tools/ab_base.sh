#!/bin/bash
# Build tools/ab/libaa_<name>.so: the in-tree library with aa_cnn.hip (and the
# conv headers) taken from git revision REV -- an A/B baseline for CNN kernel
# changes that links against the current ABI of every other source.
# usage: bash tools/ab_base.sh REV NAME
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/tools/ab/src_$NAME
rm -rf "$D"; mkdir -p "$D"
for f in aa_cnn.hip aa_conv_x3.h aa_conv_wg.h aa_common.h; do
  git -C "$ROOT" show "$REV:audio-analysis_amd/csrc/$f" > "$D/$f"
done
sed -i "s|../../include/aa.h|$ROOT/include/aa.h|" "$D/aa_common.h"
python -c "import sys; sys.path.insert(0, '$ROOT'); import __graft_entry__ as g; g.build()"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I"$ROOT/include" -mllvm -amdgpu-mfma-vgpr-form \
  -c "$D/aa_cnn.hip" -o "$D/aa_cnn.o"
OBJS=$(ls "$ROOT"/audio-analysis_amd/build/*.o | grep -v '/aa_cnn.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$D/aa_cnn.o" $OBJS -o "$ROOT/tools/ab/libaa_$NAME.so"
echo "$ROOT/tools/ab/libaa_$NAME.so"
