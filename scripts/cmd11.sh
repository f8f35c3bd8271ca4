set -u
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "double_buffered or held" > gpurun_out/pt11.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pt11.log
case $rc in 0|1) ;; *) exit $rc;; esac
WARM=150 B2B=8 timeout -k 10 300 python scripts/kstamps.py 65536x3x3,4096x16x32 > gpurun_out/kstamps11.log 2>&1; echo "kstamps rc=$?"; grep -v amdgpu.ids gpurun_out/kstamps11.log | cut -c1-700
