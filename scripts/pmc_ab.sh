#!/bin/bash
# PMC of alternative libmarlnav builds at one config: for each LIB, the
# passes in ONLY (scripts/pmc_collect.sh numbering) with --kernel-trace only,
# then a per-lib summary (gpurun_out/pmcab_<tag>_<cfg>.json).
#   LIBS="marl-nav_amd/lib/libmarlnav.so marl-nav_amd/lib/x.so" ONLY=14 bash scripts/pmc_ab.sh 4096x16x32
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${1:-4096x16x32}
PASSES=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVE_CYCLES"
 "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
 "FETCH_SIZE GRBM_GUI_ACTIVE"
 "WRITE_SIZE GRBM_GUI_ACTIVE"
 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS SQ_IFETCH"
 "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES"
 "InstrFetchLatency SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES"
)
ONLY=${ONLY:-14}
for lib in ${LIBS:-marl-nav_amd/lib/libmarlnav.so}; do
  tag=$(basename $lib .so)
  OUT=gpurun_out/pmcab_${tag}_$CFG
  mkdir -p $OUT
  i=0
  for p in "${PASSES[@]}"; do
    case "$ONLY" in *$i*) ;; *) i=$((i+1)); continue;; esac
    MARLNAV_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $p --output-format csv -d $OUT/p$i -o run -- python scripts/pmc_run.py $CFG 40 > $OUT/p$i.log 2>&1
    rc=$?; echo "$tag pass $i rc=$rc"
    case $rc in 0|1) ;; *) exit $rc;; esac
    i=$((i+1))
  done
  python scripts/pmc_summarize.py $OUT ${tag}_$CFG > /dev/null
  python - "$OUT/../pmc_${tag}_$CFG.json" "$tag" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
g = lambda k: d.get(k, float("nan"))
print(f"{sys.argv[2]:>14} us {g('kernel_us_median_under_pmc'):.2f} conflict/idx {g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):.4f} "
      f"wait/wave {g('SQ_WAIT_ANY') / max(g('SQ_WAVE_CYCLES'), 1):.3f} valu/wave {g('SQ_INSTS_VALU') / max(g('SQ_WAVES'), 1):.0f} "
      f"lds/wave {g('SQ_INSTS_LDS') / max(g('SQ_WAVES'), 1):.0f} waitlds {g('SQ_WAIT_INST_LDS'):.4g}")
if 'InstrFetchLatency' in d:
    print(f"{'':>14} ifetch latency {g('InstrFetchLatency'):.0f} cyc  wait_inst/wave {g('SQ_WAIT_INST_ANY') / max(g('SQ_WAVE_CYCLES'), 1):.3f} wait/wave {g('SQ_WAIT_ANY') / max(g('SQ_WAVE_CYCLES'), 1):.3f} wave_cycles/wave {g('SQ_WAVE_CYCLES') / max(g('SQ_WAVES'), 1):.0f}")
if 'SQC_ICACHE_MISSES' in d:
    print(f"{'':>14} icache req {g('SQC_ICACHE_REQ'):.0f} miss {g('SQC_ICACHE_MISSES'):.0f} dup {g('SQC_ICACHE_MISSES_DUPLICATE'):.0f} "
          f"tc_inst {g('SQC_TC_INST_REQ'):.0f} ifetch/wave {g('SQ_IFETCH') / max(g('SQ_WAVES'), 1):.1f}")
PY
done
