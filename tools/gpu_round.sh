#!/usr/bin/env bash
# One GPU-box pass at the current tree (run from the repo root via gpurun):
#   1. the GPU test suite (pytest -m gpu)                -> gpurun_out/<tag>/pytest.log
#   2. tools/profile.sh per config (trace + 5 PMC passes) -> gpurun_out/prof_<tag>_<cfg>/
#   3. the per-config summaries merged into one config-keyed file
#      (profiles/pmc_latest.json's shape)                -> gpurun_out/<tag>/pmc_merged.json
#   4. bench.py reading that file, so its roofline uses counters of this very
#      build                                             -> gpurun_out/<tag>/bench.json
# Steps are chained: the first failure ends the script.  gpurun_out/<tag>/command.txt
# records the command.
# usage: bash tools/gpu_round.sh <tag> [configs=c3,c5,c5d,c2] [tests|skip-tests]
set -o pipefail
TAG=${1:?tag}
CFGS=${2:-c3,c5,c5d,c2}
TESTS=${3:-tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
echo "bash tools/gpu_round.sh $TAG $CFGS $TESTS  # $(date -u +%FT%TZ)" > "$OUT/command.txt"
if [ "$TESTS" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
fi
for c in ${CFGS//,/ }; do
  steps=3; [ "$c" = c3 ] && steps=5; [ "$c" = c2 ] && steps=20
  bash tools/profile.sh "${TAG}_$c" "$c" "$steps" || exit 1
done
python3 - "$TAG" "$CFGS" <<'EOF' || exit 1
import json, sys
tag, cfgs = sys.argv[1], sys.argv[2].split(",")
m = {c: json.load(open(f"gpurun_out/prof_{tag}_{c}/pmc_summary.json")) for c in cfgs}
json.dump(m, open(f"gpurun_out/{tag}/pmc_merged.json", "w"), indent=1)
EOF
timeout -k 10 400 python -u bench.py --pmc "$OUT/pmc_merged.json" > "$OUT/bench.json" 2> "$OUT/bench.err" ||
    { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
