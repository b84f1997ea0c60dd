set -o pipefail
mkdir -p gpurun_out
ESR_DGRAD_X3=0 timeout -k 10 200 python -u tools/diag_grid.py c5:x3 > gpurun_out/diag_c5_fwdx3_bwdf32.log 2>&1
timeout -k 10 200 python -u tools/diag_grid.py c5:f32 > gpurun_out/diag_c5_f32.log 2>&1
timeout -k 10 400 python -u tools/loop_margin.py x3:x3 x3:x6 f32:f32 > gpurun_out/diag_margins.log 2>&1
