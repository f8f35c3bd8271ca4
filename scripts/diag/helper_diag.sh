#!/bin/bash
# (GPU box) scripts/diag/helper_diag.py: graph replay, stamps and one PMC pass
# of the round-4 helper-wave build with its helper off/on (16384x3x3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
L=marl-nav_amd/lib
O=gpurun_out/helper_diag; mkdir -p $O
timeout -k 10 200 python scripts/diag/helper_diag.py $L/helper.so 16384x3x3 > $O/time.txt 2>&1 || { tail $O/time.txt; exit 1; }
grep -v amdgpu.ids $O/time.txt
STAMPS=1 STAMPS_LIB=helper_st.so WARM=150 B2B=8 timeout -k 10 200 python scripts/diag/helper_diag.py $L/helper_st.so 16384x3x3 > $O/stamps.txt 2>&1 || { tail $O/stamps.txt; exit 1; }
grep -v amdgpu.ids $O/stamps.txt | cut -c1-1200
for h in 0 1; do
  k=0
  for p in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_SMEM" "SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_BRANCH"; do
    PMC_HELPER=$h timeout -k 10 120 rocprofv3 --kernel-trace --pmc $p --output-format csv -d $O/h$h/p$k -o run -- python scripts/diag/helper_diag.py $L/helper.so 16384x3x3 > $O/h${h}_p$k.log 2>&1
    rc=$?; echo "pmc helper=$h pass $k rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
    k=$((k+1))
  done
done
python scripts/census_summarize.py $O h0 h1
