export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmc_modes -o run -- python scripts/diag/launch_modes_pmc.py 16384x3x3 > gpurun_out/pmc_modes.log 2>&1 || exit 1
ls gpurun_out/pmc_modes
