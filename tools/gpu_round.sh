#!/usr/bin/env bash
# One GPU-box pass at the current tree (run from the repo root via gpurun):
#   1. the GPU test suite (pytest -m gpu)           -> gpurun_out/<tag>/pytest.log
#   2. tools/profile.sh: kernel trace + PMC passes  -> gpurun_out/prof_<tag>/
#   3. the PMC summary becomes profiles/pmc_latest.json ON THE BOX, so
#   4. bench.py's roofline uses counters of this very build -> gpurun_out/<tag>/bench.json
# Steps are chained with &&: the first failure ends the script.
# usage: bash tools/gpu_round.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
fi
bash tools/profile.sh "$TAG" c3 5 || exit 1
cp "gpurun_out/prof_$TAG/pmc_summary.json" profiles/pmc_latest.json &&
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
cat "$OUT/bench.json"
