# A/B of the persistent double-buffered N = 32 x3 conv (variant 70; 71-74 its time-split ablations) against the
# production dispatch (v1) at the config-2/3/5 grids, ablation library; bitwise check of v70 vs v1
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/${1:-x3p}_ab.log
: > $out
export ESR_AMD_LIB=$PWD/exp_lib/libesr_exp.so AB_COUT=32 AB_ROUNDS=${AB_ROUNDS:-4}
AB_B=32 AB_HW=148 AB_CIN=${AB_CIN:-64,128,160} AB_VARIANTS=${AB_VARIANTS:-1,70,71,72,73,74} AB_DIAG=71,72,73,74 \
  timeout -k 10 200 python -u tools/x3_ab.py >> $out 2>&1 || exit $?
AB_B=16 AB_HW=96 AB_CIN=128 AB_VARIANTS=1,70 timeout -k 10 100 python -u tools/x3_ab.py >> $out 2>&1 || exit $?
AB_B=8 AB_HW=172 AB_CIN=128 AB_VARIANTS=1,70 timeout -k 10 100 python -u tools/x3_ab.py >> $out 2>&1 || exit $?
