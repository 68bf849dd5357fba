#!/usr/bin/env bash
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/pytest_stackless.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03/pytest_stackless.log; [ $rc -eq 0 ] || exit 1
rm -f gpurun_out/r03/morton8_ab.log gpurun_out/r03/stackless_ab.log
bash tools/ab_libs2.sh m4 m8 gpurun_out/r03/morton8_ab.log c5 2
echo "m rc=$?"
bash tools/ab_two_builds.sh m8 gpurun_out/r03/stackless_ab.log c3,c5,c5d 0 2
echo "s rc=$?"
