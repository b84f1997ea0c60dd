# GPU run: time split of the column-tile x3 conv from the experiment library (make -C ... exp first)
set -o pipefail
mkdir -p gpurun_out
export ESR_AMD_LIB=$PWD/tools/exp/libesr_exp.so AB_VARIANTS=50,51,52,53,54 AB_DIAG=51,52,53,54 AB_ROUNDS=4 AB_REPS=20
AB_CIN=128 timeout -k 10 240 python tools/x3_ab.py > gpurun_out/x3_split_n32.log 2>&1 && \
AB_COUT=64 timeout -k 10 240 python tools/x3_ab.py > gpurun_out/x3_split_n64.log 2>&1
