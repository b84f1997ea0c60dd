# round 4: N = 64 x3 conv tile choice at more grids (variants 1 = N split where under-filled, 65 = 12 columns, 50 = 16)
set -o pipefail
mkdir -p gpurun_out
L=$PWD/exp_lib/libesr_exp.so
for g in "8 154" "8 128" "4 96" "2 64"; do
  set -- $g
  ESR_AMD_LIB=$L AB_COUT=64 AB_CIN=200 AB_B=$1 AB_HW=$2 AB_VARIANTS=1,65,50 timeout -k 10 200 python3 tools/x3_ab.py >> gpurun_out/r4ak_n64.log 2>&1 || exit $?
done
