#!/usr/bin/env bash
# L1 (TCP) accesses and misses-to-L2 of the scene kernel for one config (own --pmc pass):
#   bash tools/pmc_l1.sh <config> <outdir>
set -o pipefail
CFG=${1:-c3}; OUT=${2:-gpurun_out/pmc_l1_$CFG}
ROOT=$(pwd)
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -T --output-format csv \
    -d "$ROOT/$OUT" -o run --kernel-include-regex scene_kernel -- python3 "$ROOT/bench.py" --steps 2 \
    --warmup 1 --config "$CFG" --cpu-baseline off --secondary= > "$ROOT/$OUT/run.log" 2>&1
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
a, m = avg.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0), avg.get("TCP_TCC_READ_REQ_sum", 0)
print({"per_dispatch": avg, "l1_read_miss_per_access": m / a if a else None})
PY
exit $rc
