#!/usr/bin/env bash
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_parity.py tests/test_gpu_progressive.py \
    -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/pytest_sort.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03/pytest_sort.log
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
RT_SORT=0 timeout -k 10 200 python -u tools/variants.py --configs c5,c5d --variants 0 --rounds 5 | sed "s/^/off /" >> gpurun_out/r03/sort_ab.log
RT_SORT=1 timeout -k 10 200 python -u tools/variants.py --configs c5,c5d --variants 0 --rounds 5 | sed "s/^/on /" >> gpurun_out/r03/sort_ab.log
done
echo "ab done"
