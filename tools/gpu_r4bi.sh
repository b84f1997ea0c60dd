# round 4: config-3 kernel view with HR_conv1's data gradient on esr_dfirst_fwd_padded (default) and without
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/torch_prof_train.py --device > gpurun_out/r4bi_on.log 2>&1 || exit $?
ESR_HR1_DFIRST=0 timeout -k 10 300 python -u tools/torch_prof_train.py --device > gpurun_out/r4bi_off.log 2>&1 || exit $?
