#!/usr/bin/env bash
# SQ counter pass of the bench for two settings of an environment variable:
#   bash tools/pmc_ab.sh <tag> <config> VAR=a VAR=b ...
# -> gpurun_out/pmcab_<tag>/<setting>/ (tools/pmc_traffic.py counters)
set -o pipefail
TAG=$1; CFG=$2; shift 2
ROOT=$(pwd)
export TMPDIR=/tmp
for SET in "$@"; do
  OUT=$ROOT/gpurun_out/pmcab_$TAG/${SET//=/_}
  mkdir -p "$OUT"
  (cd /tmp && env $SET timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE -T \
      --output-format csv -d "$OUT/sq" -o run --kernel-include-regex scene_kernel \
      -- python3 $ROOT/bench.py --steps 3 --warmup 1 --config $CFG --cpu-baseline off --secondary= > "$OUT/sq.log" 2>&1) || exit 1
  python3 - "$OUT" <<'PY'
import json, sys
sys.path.insert(0, "tools")
from pmc_traffic import counters
c = counters(sys.argv[1] + "/sq")
print(sys.argv[1], json.dumps({k: v[0] for k, v in c.items()}))
PY
done
