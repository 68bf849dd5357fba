#!/usr/bin/env bash
# Round-6 GPU steps (run from the repo root via gpurun), chained: the first
# failure ends the script.  usage: bash tools/r6_gpu.sh <out dir> <step>...
#   tests          the GPU suite on the in-tree library (sentinel-filled frames)
#   ab:<cfgs>:<reps>:<libs,...>   tools/ab_libs.sh over abl/librt_<lib>.so
#   parity:<lib>   a parity subset with RT_AMD_LIB=abl/librt_<lib>.so
#   pmcpack:<cfg>  counter passes with the leaf lists packed and not (RT_LEAF_PACK)
#   pmcphase:<cfg> counter passes of the config's frames with and without shadow rays
#   pmcl2:<lib>:<cfg>  L2 hits / misses and the TD's L1 stall of a library
#   pmcsq:<lib>:<cfg>  issue counters (SALU, VALU, branch, vector reads) of a library
set -o pipefail
OUT=${1:?out}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
  echo "== $step $(date -u +%T)"
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
          -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
      tail -2 "$OUT/pytest.log" ;;
    ab:*)
      IFS=: read -r _ cfgs reps libs <<< "$step"
      bash tools/ab_libs.sh "$OUT/ab_${libs//,/_}.log" "$cfgs" "$reps" ${libs//,/ } || exit 1
      python tools/ab_summary.py "$OUT/ab_${libs//,/_}.log" || exit 1 ;;
    parity:*)
      lib=${step#parity:}
      RT_AMD_LIB=$PWD/abl/librt_$lib.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
          --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_gpu_variants.py \
          -k "scene_bit_exact or c3_full_frame or c5_deep or c5_full or sorted_rounds or lds_staging or camera_cases" \
          > "$OUT/parity_$lib.log" 2>&1 || { tail -30 "$OUT/parity_$lib.log"; exit 1; }
      tail -2 "$OUT/parity_$lib.log" ;;
    pmcpack:*)
      # C5d (or the named config) with the leaf lists back to back vs
      # line-packed: L2 hits / misses, the TD's L1 stall, L1 waits per request
      cfg=${step#pmcpack:}
      for p in 0 1; do
        RT_LEAF_PACK=$p bash tools/pmc_probe.sh "${OUT#gpurun_out/}/pk_${cfg}_p${p}_a" "$cfg" 0 \
            TCC_HIT_sum TCC_MISS_sum TD_TC_STALL_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE || exit 1
        RT_LEAF_PACK=$p bash tools/pmc_probe.sh "${OUT#gpurun_out/}/pk_${cfg}_p${p}_b" "$cfg" 0 \
            TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum \
            GRBM_GUI_ACTIVE || exit 1
      done
      python3 tools/pmc_probe_sum.py "$OUT"/pk_${cfg}_p* > "$OUT/pmc_pack_$cfg.json" || exit 1 ;;
    pmcphase:*)
      # the same frames with and without their shadow rays: which walks miss the L2
      cfg=${step#pmcphase:}
      for ph in all prim; do
        ex=""; [ $ph = prim ] && ex="--no-shadows"
        PROBE_EXTRA=$ex bash tools/pmc_probe.sh "${OUT#gpurun_out/}/ph_${cfg}_${ph}_a" "$cfg" 0 \
            TCC_HIT_sum TCC_MISS_sum TD_TC_STALL_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE || exit 1
        PROBE_EXTRA=$ex bash tools/pmc_probe.sh "${OUT#gpurun_out/}/ph_${cfg}_${ph}_b" "$cfg" 0 \
            TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum \
            GRBM_GUI_ACTIVE || exit 1
        PROBE_EXTRA=$ex bash tools/pmc_probe.sh "${OUT#gpurun_out/}/ph_${cfg}_${ph}_c" "$cfg" 0 \
            SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE || exit 1
      done
      python3 tools/pmc_probe_sum.py "$OUT"/ph_${cfg}_* > "$OUT/pmc_phase_$cfg.json" || exit 1 ;;
    pmcl2:*)
      IFS=: read -r _ lib cfg <<< "$step"
      RT_AMD_LIB=$PWD/abl/librt_$lib.so bash tools/pmc_probe.sh "${OUT#gpurun_out/}/l2_${lib}_$cfg" "$cfg" 0 \
          TCC_HIT_sum TCC_MISS_sum TD_TC_STALL_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE || exit 1
      python3 tools/pmc_probe_sum.py "$OUT/l2_${lib}_$cfg" > "$OUT/pmc_l2_${lib}_$cfg.json" || exit 1 ;;
    pmcsq:*)
      # issue counters of the timed kernel for a library (abl/librt_<lib>.so) and config
      IFS=: read -r _ lib cfg <<< "$step"
      RT_AMD_LIB=$PWD/abl/librt_$lib.so bash tools/pmc_probe.sh "${OUT#gpurun_out/}/sq_${lib}_$cfg" "$cfg" 0 \
          SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAVES \
          GRBM_GUI_ACTIVE || exit 1
      python3 tools/pmc_probe_sum.py "$OUT/sq_${lib}_$cfg" > "$OUT/pmc_sq_${lib}_$cfg.json" || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
