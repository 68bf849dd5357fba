#!/usr/bin/env bash
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/pytest_dense1.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03/pytest_dense1.log; [ $rc -eq 0 ] || exit 1
rm -f gpurun_out/r03/dense1_ab.log
for i in 1 2 3; do
RT_DENSE1=0 timeout -k 10 200 python -u tools/variants.py --configs c3 --variants 0 --rounds 7 | sed "s/^/off /" >> gpurun_out/r03/dense1_ab.log
RT_DENSE1=1 timeout -k 10 200 python -u tools/variants.py --configs c3 --variants 0 --rounds 7 | sed "s/^/on /" >> gpurun_out/r03/dense1_ab.log
done
echo "ab done"
