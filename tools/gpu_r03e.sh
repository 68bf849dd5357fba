#!/usr/bin/env bash
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 200 python -u -m pytest tests/test_gpu_variants.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/pytest_batch2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r03/pytest_batch2.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/variants.py --configs c3,c5 --variants 0:0::63,0:0::16,0:0::62 --rounds 5 > gpurun_out/r03/refill_ab3.log 2>&1
echo "ab rc=$?"
RT_BATCH_W7=1 timeout -k 10 300 python -u tools/variants.py --configs c3,c5 --variants 0:0::63,0:0::16 --rounds 5 > gpurun_out/r03/refill_ab3_w7.log 2>&1
echo "ab7 rc=$?"
