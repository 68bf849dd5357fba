#!/usr/bin/env bash
# Alternating-process A/B of prebuilt libraries abl/librt_<name>.so (made by
# tools/build_exp.sh from the working tree, or tools/build_rev.sh from a git
# revision), interleaved per repetition so clock drift hits all of them alike.
# Run on the GPU box from the repo root.  The log's first line is the command
# that made it (profiles/r04 convention).
#
# usage: bash tools/ab_libs.sh <log> <configs> <reps> <name>...
#   TOOL=variants (default): tools/variants.py plain frames of <configs>
#   TOOL=share:              tools/share_cost.py (1/8 C3 tile share + full frame)
#   ENV="A=1 B=2":           extra environment for every run (e.g. RT_SORT=0)
#   e.g. bash tools/ab_libs.sh gpurun_out/r04/node_ab.log c3,c5,c5d 3 base dword
set -e -o pipefail
LOG=${1:?log}; CFGS=${2:?configs}; REPS=${3:?reps}; shift 3
[ $# -ge 1 ] || { echo "name at least one build" >&2; exit 2; }
TOOL=${TOOL:-variants}
export TMPDIR=/tmp
mkdir -p "$(dirname "$LOG")"
echo "# cmd: TOOL=$TOOL ENV='${ENV:-}' bash tools/ab_libs.sh $LOG $CFGS $REPS $*" >> "$LOG"
for i in $(seq "$REPS"); do
  for L in "$@"; do
    case $TOOL in
      variants)
        env ${ENV:-} RT_AMD_LIB=$PWD/abl/librt_$L.so timeout -k 10 200 python tools/variants.py \
            --configs "$CFGS" --variants 0 --rounds 5 | sed "s/^/$L /" >> "$LOG" ;;
      share)
        env ${ENV:-} RT_AMD_LIB=$PWD/abl/librt_$L.so timeout -k 10 120 python tools/share_cost.py \
            2>/dev/null | sed "s/^/$L /" >> "$LOG" ;;
      *) echo "unknown TOOL=$TOOL" >&2; exit 2 ;;
    esac
  done
done
