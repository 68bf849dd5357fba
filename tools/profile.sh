#!/usr/bin/env bash
# Profile the headline bench on the GPU box (run from the repo root via gpurun):
#   1. rocprofv3 --kernel-trace --stats  (per-kernel durations)
#   2. rocprofv3 --pmc FETCH_SIZE        (own pass)
#   3. rocprofv3 --pmc WRITE_SIZE        (own pass)
#   4. rocprofv3 --pmc SQ_WAVES,SQ_INSTS_VALU,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_INSTS_SALU,
#      SQ_INSTS_BRANCH,SQ_THREAD_CYCLES_VALU,SQ_WAIT_ANY,GRBM_GUI_ACTIVE (8 SQ + 1 GRBM)
#   5. rocprofv3 --pmc TA_TA_BUSY_sum,TD_TD_BUSY_sum,TD_TC_STALL_sum,GRBM_GUI_ACTIVE
#      (the vector-memory return path: 1 TA + 2 TD + 1 GRBM)
# then tools/pmc_traffic.py -> gpurun_out/prof_<tag>/pmc_summary.json
# Every GPU step has its own time limit and the steps are chained with &&.
set -o pipefail
TAG=${1:-r01}
CFG=${2:-c3}
STEPS=${3:-3}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps $STEPS --warmup 1 --config $CFG --cpu-baseline off --secondary="
cd /tmp || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run \
    -- python3 $BENCH > "$OUT/trace.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT/fetch" -o run \
    --kernel-include-regex scene_kernel -- python3 $BENCH > "$OUT/fetch.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT/write" -o run \
    --kernel-include-regex scene_kernel -- python3 $BENCH > "$OUT/write.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE -T \
    --output-format csv -d "$OUT/sq" -o run --kernel-include-regex scene_kernel \
    -- python3 $BENCH > "$OUT/sq.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE -T \
    --output-format csv -d "$OUT/vmem" -o run --kernel-include-regex scene_kernel \
    -- python3 $BENCH > "$OUT/vmem.log" 2>&1 &&
cd "$ROOT" && python3 tools/pmc_traffic.py "$OUT" "$CFG" > "$OUT/pmc_summary.json"
rc=$?
echo "profile rc=$rc"
exit $rc
