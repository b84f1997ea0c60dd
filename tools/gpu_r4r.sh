# round 4: N=32 x3 conv at config 5's grids (B=8 x 172^2 / 154^2) and a small grid: automatic vs 12-column tiles
set -o pipefail
mkdir -p gpurun_out
ESR_AMD_LIB=$PWD/exp_lib/libesr_exp.so AB_B=8 AB_HW=172,154,64 AB_VARIANTS=1,64 timeout -k 10 200 python3 tools/x3_ab.py > gpurun_out/r4r_x3ab_c5.log 2>&1
