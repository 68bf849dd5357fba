#!/usr/bin/env bash
# One rocprofv3 --pmc pass over the TIMED scene kernel (scene_kernel_w8) of a
# few plain frames (tools/write_probe.py), from the repo root via gpurun:
#   bash tools/pmc_probe.sh <outdir> <config> <chunk field 0..4> <counters...>
# Output: gpurun_out/<outdir>/ (rocprofv3 csv + log); summarise with
# tools/pmc_probe_sum.py.  Each pass has its own time limit; a refused or
# failing counter set fails the pass (the caller chains passes with &&).
# PROBE_EXTRA: more write_probe.py arguments (e.g. --no-shadows).
set -o pipefail
D=${1:?outdir}; CFG=${2:?config}; CH=${3:?chunk}; shift 3
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$D
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
echo "pmc_probe $D $CFG chunk=$CH: $*" > "$OUT/command.txt"
timeout -s KILL 240 rocprofv3 --pmc "$@" -T --output-format csv -d "$OUT" -o run \
    --kernel-include-regex scene_kernel_w8 -- \
    python3 "$ROOT/tools/write_probe.py" --config "$CFG" --chunk "$CH" --frames 3 ${PROBE_EXTRA:-} > "$OUT/probe.log" 2>&1
rc=$?
echo "pmc_probe $D rc=$rc"
exit $rc
