#!/usr/bin/env bash
# A/B of several builds (abl/librt_<name>.so from tools/build_rev.sh, or
# copies of the in-tree library), interleaved per repetition so drift hits all
# of them alike.  Run on the GPU box from the repo root (build_ab must not be
# in .gpurunignore for that call).
# usage: bash tools/ab_libs.sh <log> <configs> <reps> <name>...
#   e.g. bash tools/ab_libs.sh gpurun_out/leaf_chunk_ab.log c3,c5 3 base ck3 ck4
set -e -o pipefail
LOG=${1:?log}; CFGS=${2:?configs}; REPS=${3:?reps}; shift 3
[ $# -ge 1 ] || { echo "name at least one build" >&2; exit 2; }
export TMPDIR=/tmp
mkdir -p "$(dirname "$LOG")"
for i in $(seq "$REPS"); do
  for L in "$@"; do
    RT_AMD_LIB=abl/librt_$L.so timeout -k 10 200 python tools/variants.py --configs "$CFGS" \
        --variants 0 --rounds 5 | sed "s/^/$L /" >> "$LOG"
  done
done
