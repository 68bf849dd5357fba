#!/usr/bin/env bash
# Round-3 check after the per-config leaf capacity (C3, C4, C5 at 12): GPU suite, C3, C5, C5d
# and C2 profiles merged into one config-keyed summary (profiles/pmc_latest.json's
# shape), then the bench reading that summary.
# usage: bash tools/gpu_r03b.sh <tag>
set -o pipefail
TAG=${1:-r03n}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc"
tail -3 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
bash tools/profile.sh "${TAG}_c3" c3 5 && bash tools/profile.sh "${TAG}_c5" c5 3 &&
bash tools/profile.sh "${TAG}_c5d" c5d 3 && bash tools/profile.sh "${TAG}_c2" c2 20 &&
python3 - "$TAG" <<'EOF' &&
import json, sys
tag = sys.argv[1]
m = {c: json.load(open(f"gpurun_out/prof_{tag}_{c}/pmc_summary.json")) for c in ("c3", "c5", "c5d", "c2")}
json.dump(m, open(f"gpurun_out/{tag}/pmc_merged.json", "w"), indent=1)
EOF
timeout -k 10 300 python -u bench.py --pmc "$OUT/pmc_merged.json" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
echo "bench rc=$rc"
cat "$OUT/bench.json"
exit $rc
