# round 4: N=32 x3 conv at config 3's grid (B=16 x 96^2): automatic (8-row classic) vs 12-column tiles, per launch and
# in the training step
set -o pipefail
mkdir -p gpurun_out
ESR_AMD_LIB=$PWD/exp_lib/libesr_exp.so AB_B=16 AB_HW=96 AB_VARIANTS=1,64,26,50 timeout -k 10 200 python3 tools/x3_ab.py > gpurun_out/r4q_x3ab96.log 2>&1 || exit $?
bash tools/gpu_ab_env.sh ESR_X3_KERNEL 1 64 || exit $?
