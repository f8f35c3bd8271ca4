#!/bin/bash
# PMC passes (counters only with --kernel-trace; never with sys/runtime traces)
# over scripts/pmc_run.py; summary -> gpurun_out/pmc_<cfg>.json
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${1:-65536x3x3}
OUT=gpurun_out/pmc_$CFG
mkdir -p $OUT
PASSES=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVE_CYCLES"
 "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
 "FETCH_SIZE GRBM_GUI_ACTIVE"
 "WRITE_SIZE GRBM_GUI_ACTIVE"
 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS SQ_IFETCH"
)
ONLY=${ONLY:-01234}   # which passes to run
i=0
for p in "${PASSES[@]}"; do
  case "$ONLY" in *$i*) ;; *) i=$((i+1)); continue;; esac
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $p --output-format csv -d $OUT/p$i -o run -- python scripts/pmc_run.py $CFG 40 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 0|1) ;; *) exit $rc;; esac
  i=$((i+1))
done
python scripts/pmc_summarize.py $OUT $CFG
