set -o pipefail
mkdir -p gpurun_out
export AB_ROUNDS=4 AB_REPS=20 ESR_AMD_LIB=$PWD/tools/exp/libesr_exp.so
AB_COUT=64 AB_CIN=192 AB_HW=148,96 AB_VARIANTS=1,50,55,56,57 AB_DIAG=56,57 timeout -k 10 300 python tools/x3_ab.py > gpurun_out/ab4_n64.log 2>&1 ; \
AB_COUT=32 AB_CIN=64,128 AB_HW=148,96 AB_VARIANTS=1,50,55,56,57 AB_DIAG=56,57 timeout -k 10 300 python tools/x3_ab.py > gpurun_out/ab4_n32.log 2>&1
