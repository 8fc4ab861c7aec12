#!/bin/bash
# Build libgpscore.so from a git ref (default HEAD) into ab/libgpscore_<name>.so, here in the
# container, so a same-box A/B on the GPU (tools/ab_lib.sh) can load it beside the working lib.
#   bash tools/build_ref_lib.sh HEAD base
set -e
REF=${1:-HEAD}; NAME=${2:-base}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/gps_ref_$NAME
rm -rf $W; git -C $ROOT worktree prune
git -C $ROOT worktree add --detach $W $REF >/dev/null
mkdir -p $ROOT/ab
make -s -C $W/scoring-rules-for-gaussian-process-regression-a-new-approach-to-inference_amd/csrc -j8 \
  GPS_BUILD_DIR=/tmp/gps_ref_build_$NAME GPS_LIB_OUT=$ROOT/ab/libgpscore_$NAME.so
git -C $ROOT worktree remove --force $W
echo "built ab/libgpscore_$NAME.so from $REF"
