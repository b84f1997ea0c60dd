set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_zopt_overflow.py > gpurun_out/diag_zopt.log 2>&1
timeout -k 10 400 python -u tools/diag_grid.py c3:f32 c5:x3 > gpurun_out/diag_grid.log 2>&1
