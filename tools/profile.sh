#!/usr/bin/env bash
# Profile the bench's scene kernel for one config on the GPU box (run from the
# repo root via gpurun).  One rocprofv3 run per pass, each under its own time
# limit, chained with &&:
#   1. --kernel-trace --stats                (per-kernel durations)
#   2. --pmc FETCH_SIZE                      (own pass: 3 TCC slots)
#   3. --pmc WRITE_SIZE                      (own pass: 2 TCC slots)
#   4. --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU
#            SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE  (8 SQ + 1 GRBM)
#   5. --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
#            (the vector-memory return path: 1 TA + 2 TD + 1 GRBM)
#   6. --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TA_FLAT_READ_WAVEFRONTS_sum
#            TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE
#            (vector-memory instructions and L1 accesses per launch: the
#             charged bytes of bench.py's roofline.waste; 2 SQ + 1 TA + 1 TCP + 1 GRBM)
# then tools/pmc_traffic.py -> gpurun_out/prof_<tag>/pmc_summary.json.
# usage: bash tools/profile.sh <tag> [config=c3] [steps=3] [extra bench args]
set -o pipefail
TAG=${1:-r04}
CFG=${2:-c3}
STEPS=${3:-3}
EXTRA=${4:-}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
echo "bash tools/profile.sh $TAG $CFG $STEPS '$EXTRA'  # $(date -u +%FT%TZ)" > "$OUT/command.txt"
export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps $STEPS --warmup 1 --config $CFG --cpu-baseline off --secondary= $EXTRA"
cd /tmp || exit 1
pmc() {  # pmc <dir> <counters...>: one --pmc pass on the scene kernel
  local d=$1; shift
  timeout -k 10 400 rocprofv3 --pmc "$@" -T --output-format csv -d "$OUT/$d" -o run \
      --kernel-include-regex scene_kernel -- python3 $BENCH > "$OUT/$d.log" 2>&1
}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o run \
    -- python3 $BENCH > "$OUT/trace.log" 2>&1 &&
pmc fetch FETCH_SIZE &&
pmc write WRITE_SIZE &&
pmc sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_BRANCH \
    SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE &&
pmc vmem TA_TA_BUSY_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE &&
pmc vinst SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum \
    GRBM_GUI_ACTIVE &&
cd "$ROOT" && python3 tools/pmc_traffic.py "$OUT" "$CFG" > "$OUT/pmc_summary.json"
rc=$?
echo "profile $TAG $CFG rc=$rc"
exit $rc
