#!/usr/bin/env bash
# Deeper PMC passes on the scene kernel (one counter group per rocprofv3 pass).
# usage: bash tools/pmc_deep.sh <tag> [config] [extra bench args] [set: sq|mem]
#        (from the repo root, via gpurun)
# A pass whose counters are rejected just fails; a timeout/crash stops the script.
TAG=${1:-deep}; CFG=${2:-c3}; EXTRA=${3:-}; SET=${4:-sq}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps 2 --warmup 0 --config $CFG --cpu-baseline off --secondary= $EXTRA"
cd /tmp || exit 1
i=0
while read -r COUNTERS; do
  [ -z "$COUNTERS" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $COUNTERS -T --output-format csv -d "$OUT/p$i" -o run \
      --kernel-include-regex scene_kernel -- python3 $BENCH > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i [$COUNTERS] rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
done < <(if [ "$SET" = mem ]; then cat <<'LIST'
TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE
TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES
SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TD_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum
LIST
else cat <<'LIST'
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_LEVEL_WAVES SQ_CYCLES
TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCP_TCC_READ_REQ_sum
LIST
fi)
cd "$ROOT" && python3 - "$OUT" <<'PY'
import csv, glob, json, os, sys
from collections import defaultdict
out = sys.argv[1]; res = {}
for path in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(path)):
        per[r["Counter_Name"]][r.get("Dispatch_Id")] += float(r["Counter_Value"])
    for k, v in per.items():
        res[k] = sum(v.values()) / len(v)
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
PY
