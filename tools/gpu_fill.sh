# x3 conv time split at the config-2 trunk shapes (B=32, 148² = 128² + the CEM pre-pad, the production column-tile kernel): full (1, 50) vs
# LDS-DMA of chunk 0 only (51), no fragment reads / MFMAs (52), no epilogue stores (53), 51+53 (54); experiment build
# needs the experiment library in the GPU snapshot: make -C explorable-super-resolution_old_amd/csrc exp EXP_OUT=../../exp_lib/libesr_exp.so, and drop ./exp_lib from .gpurunignore for the run
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/x3_fill.log
: > $out
export ESR_AMD_LIB=$PWD/exp_lib/libesr_exp.so AB_HW=148 AB_VARIANTS=1,50,51,52,53,54 AB_DIAG=51,52,53,54 AB_ROUNDS=4
AB_COUT=32 AB_CIN=64,128,160 timeout -k 10 240 python -u tools/x3_ab.py >> $out 2>&1 && \
AB_COUT=64 AB_CIN=192 timeout -k 10 240 python -u tools/x3_ab.py >> $out 2>&1
