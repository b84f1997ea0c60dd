# round 4: N = 64 x3 convs in 12-column tiles (ablation variant 65) vs the N split (1) vs 16-column tiles (50)
set -o pipefail
mkdir -p gpurun_out
L=$PWD/exp_lib/libesr_exp.so
ESR_AMD_LIB=$L AB_COUT=64 AB_CIN=200 AB_B=16 AB_HW=96 AB_VARIANTS=1,65,50 timeout -k 10 200 python3 tools/x3_ab.py > gpurun_out/r4aj_n64.log 2>&1 || exit $?
ESR_AMD_LIB=$L AB_COUT=64 AB_CIN=200 AB_B=8 AB_HW=172 AB_VARIANTS=1,65,50 timeout -k 10 200 python3 tools/x3_ab.py >> gpurun_out/r4aj_n64.log 2>&1 || exit $?
ESR_AMD_LIB=$L AB_COUT=64 AB_CIN=192 AB_B=32 AB_HW=148 AB_VARIANTS=1,65 timeout -k 10 200 python3 tools/x3_ab.py >> gpurun_out/r4aj_n64.log 2>&1 || exit $?
bash tools/gpu_ab_env.sh ESR_X3_KERNEL 1 65 || exit $?
