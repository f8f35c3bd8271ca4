export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/wt_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/wt_pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/wt_pytest.log | head; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
for c in 1024x3x8 2x3x3 8192x3x3; do for l in libmarlnav.so ref.so; do echo "== $l"; MARLNAV_LIB=marl-nav_amd/lib/$l timeout -k 10 200 python scripts/diag/launch_modes.py $c 200 2>&1 | grep -v amdgpu.ids | grep -v -E "side" || exit 1; done; done
