#!/usr/bin/env bash
# L2 hit rate of the scene kernel for one config (own --pmc pass, run from the repo root on the GPU box):
#   bash tools/pmc_l2.sh <config> <outdir>
set -o pipefail
CFG=${1:-c3}; OUT=${2:-gpurun_out/pmc_l2_$CFG}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T --output-format csv -d "$ROOT/$OUT" -o run \
    --kernel-include-regex scene_kernel -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --config "$CFG" \
    --cpu-baseline off --secondary= > "$ROOT/$OUT/run.log" 2>&1
rc=$?
cd "$ROOT" && python3 - "$OUT" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
per = defaultdict(lambda: defaultdict(float))
for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(p)):
        per[r["Counter_Name"]][r.get("Dispatch_Id")] += float(r["Counter_Value"])
avg = {k: sum(v.values()) / len(v) for k, v in per.items() if v}
h, m = avg.get("TCC_HIT_sum", 0), avg.get("TCC_MISS_sum", 0)
print({"per_dispatch": avg, "l2_hit_rate": h / (h + m) if h + m else None})
PY
exit $rc
