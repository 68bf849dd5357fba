#!/usr/bin/env bash
# C5d at leaf capacity 10: its whole-frame parity test, a fresh PMC entry
# merged into the committed summary (other configs unchanged), the bench.
set -o pipefail
OUT=gpurun_out/r03p
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread \
    -p no:cacheprovider -k "c5_deep_full_frame" > "$OUT/pytest_c5d.log" 2>&1 || { tail -30 "$OUT/pytest_c5d.log"; exit 1; }
tail -1 "$OUT/pytest_c5d.log"
bash tools/profile.sh r03p_c5d c5d 3 || exit 1
python3 - <<'P' &&
import json
m = json.load(open("profiles/pmc_latest.json"))
m["c5d"] = json.load(open("gpurun_out/prof_r03p_c5d/pmc_summary.json"))
json.dump(m, open("gpurun_out/r03p/pmc_merged.json", "w"), indent=1)
P
timeout -k 10 300 python -u bench.py --pmc "$OUT/pmc_merged.json" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['value']); c=d['secondary']['c5d']; print('c5d', c['kernel_ms'], c['roofline']['bound'], c['roofline']['frac'], c.get('depth_reached'))"
