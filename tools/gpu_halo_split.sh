# time split of the discriminator's x3 halo kernel at the config-3 shapes (experiment build): full (0), no weight-slab
# staging (1), no fragment reads / MFMAs (2), halo window staged once (4), 1+4 (5)
# needs the experiment library in the GPU snapshot: make -C explorable-super-resolution_old_amd/csrc exp EXP_OUT=../../exp_lib/libesr_exp.so, and drop ./exp_lib from .gpurunignore for the run
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/halo_split.log
: > $out
export ESR_AMD_LIB=$PWD/exp_lib/libesr_exp.so AB_LAYERS=conv0_1,conv1_0,conv1_1,conv2_0 AB_TAGS=x3_halo
for d in 0 1 2 4 5 0; do
  echo "== ESR_HALO_DBG=$d" >> $out
  ESR_HALO_DBG=$d timeout -k 10 200 python -u tools/dconv_ab.py 2>&1 | grep '{' >> $out || exit $?
done
