#!/bin/bash
# (GPU box) Per-phase dynamic instruction census of the step kernel
# (VERDICT r4 item 1a): three PMC passes (counters with --kernel-trace only)
# over scripts/pmc_run.py for each library build given, e.g. the kernel
# truncation builds of scripts/build_variant.sh (AB 4096 entry, 8192 staged,
# 16384 observed, 2 all but the block store) and the full kernel; the
# per-phase shares are the differences (scripts/census_summarize.py).
#   (PMC_SET=fetch: instruction-fetch and I-cache counters instead)
#   CFG=65536x3x3 bash scripts/valu_census.sh full:marl-nav_amd/lib/libmarlnav.so ab2:marl-nav_amd/lib/ab2.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${CFG:-65536x3x3}
PASSES=(
 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVE_CYCLES"
 "SQ_WAVES SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"
 "SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES"
)
if [ "${PMC_SET:-}" = fetch ]; then  # instruction-fetch census (code size, I-cache)
PASSES=(
 "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_IFETCH"
 "SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
)
fi
for spec in "$@"; do
  tag=${spec%%:*}; lib=${spec#*:}
  OUT=gpurun_out/census_${CFG}/$tag
  rm -rf $OUT; mkdir -p $OUT
  i=0
  for p in "${PASSES[@]}"; do
    MARLNAV_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $p --output-format csv -d $OUT/p$i -o run -- python scripts/pmc_run.py $CFG 40 > $OUT/p$i.log 2>&1
    rc=$?; echo "$tag pass $i rc=$rc"
    case $rc in 0|1) ;; *) exit $rc;; esac
    i=$((i+1))
  done
done
python scripts/census_summarize.py gpurun_out/census_${CFG} "$@"
