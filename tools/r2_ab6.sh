set -o pipefail
mkdir -p gpurun_out
export AB_ROUNDS=4 AB_REPS=20
AB_COUT=32 AB_CIN=64,96,128,160 AB_HW=148,96 AB_VARIANTS=1,61,24 timeout -k 10 300 python tools/x3_ab.py > gpurun_out/ab6_n32.log 2>&1
