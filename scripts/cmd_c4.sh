# parity suite + per-phase stamps of the small/stress configs
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pt.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 120 python scripts/kstamps.py ${CFGS:-4096x16x32,1024x3x8} > gpurun_out/kst_c4.log 2>&1
