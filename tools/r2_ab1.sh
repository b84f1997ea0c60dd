set -o pipefail
mkdir -p gpurun_out
export AB_ROUNDS=4 AB_REPS=20
AB_COUT=64 AB_CIN=192 AB_HW=148 AB_VARIANTS=1,40,41,45,42,43,44,46 AB_DIAG=42,43,44,46 timeout -k 10 300 python tools/x3_ab.py > gpurun_out/ab1_n64.log 2>&1 && \
AB_COUT=32 AB_CIN=128 AB_HW=148 AB_VARIANTS=1,22,40,41,42,43,44 AB_DIAG=42,43,44 timeout -k 10 300 python tools/x3_ab.py > gpurun_out/ab1_n32.log 2>&1
