#!/usr/bin/env bash
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_parity.py -k "sorted or c5 or partial or bit_exact or progressive" \
    -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/pytest_morton8.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r03/pytest_morton8.log; [ $rc -eq 0 ] || exit 1
rm -f gpurun_out/r03/morton8_ab.log
bash tools/ab_libs2.sh m4 m8 gpurun_out/r03/morton8_ab.log c5 3
echo "ab rc=$?"
