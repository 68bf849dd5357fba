#!/usr/bin/env bash
# Round-3 closing check: smoke, the whole GPU suite, the bench line (PMC from
# profiles/pmc_latest.json), and a C2 leaf-capacity sweep.
set -o pipefail
OUT=gpurun_out/r03o
mkdir -p "$OUT"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['value'], d['roofline']['bound'], d['roofline']['frac'])"
timeout -k 10 200 python -u tools/variants.py --configs c2 --variants 0:0::8,0:0::4,0:0::12,0:0::16 --rounds 15 > "$OUT/c2_cap.log" 2>&1 && cat "$OUT/c2_cap.log"
