#!/usr/bin/env bash
# Round-3 check on one GPU box: GPU suite, C3 + C5 profiles, bench.
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r03/pytest_gpu.log 2>&1
echo "pytest rc=$?"
tail -3 gpurun_out/r03/pytest_gpu.log
bash tools/profile.sh r03_c3 c3 5 && bash tools/profile.sh r03_c5 c5 3 &&
timeout -k 10 300 python -u bench.py --pmc gpurun_out/prof_r03_c3/pmc_summary.json > gpurun_out/r03/bench.json 2> gpurun_out/r03/bench.err
echo "bench rc=$?"
