#!/usr/bin/env bash
# Alternating-process A/B/... of prebuilt libraries abl/librt_<name>.so
# usage: bash tools/ab_libsn.sh <log> <configs> <reps> <name> <name> [<name> ...]
set -e -o pipefail
LOG=${1:?log}; CFGS=${2:?configs}; REPS=${3:?reps}; shift 3
export TMPDIR=/tmp
for i in $(seq "$REPS"); do
  for L in "$@"; do
    RT_AMD_LIB=$PWD/abl/librt_$L.so timeout -k 10 200 python tools/variants.py --configs "$CFGS" \
        --variants 0 --rounds 5 | sed "s/^/$L /" >> "$LOG"
  done
done
