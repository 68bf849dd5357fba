#!/usr/bin/env bash
# batched rounds + shadow refill: parity, then same-process A/B of the refill threshold
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_parity.py tests/test_gpu_progressive.py \
    -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/pytest_batch.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03/pytest_batch.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/variants.py --configs c3,c5,c5d --variants 0:0::63,0:0::8,0:0::16,0:0::32,0:0::48 --rounds 5 \
    > gpurun_out/r03/refill_ab.log 2>&1
echo "ab rc=$?"
