#!/usr/bin/env bash
# Closing check at the current tree (run from the repo root via gpurun): the GPU
# test suite, smoke(), the default bench line, and a rocprofv3 kernel trace of
# the headline bench (C3 only) whose average scene-kernel duration must agree
# with the bench line's HIP-event kernel_ms.  Outputs under $OUT (default gpurun_out/closing/).
# usage: bash tools/closing_check.sh
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/closing}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -n 3 $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 5 --secondary '' --cpu-baseline off > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { tail -20 $OUT/bench_prof.err; exit 1; }
find $OUT/prof -name '*kernel_stats*' | head
