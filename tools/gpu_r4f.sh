# round-4 diagnostics: C3 grid parity vs the generator's backward precision; the C5 first timed iteration vs the
# headline's step count; config-3 kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/grid_c3_ab.py base dgrad_f32 wgrad_f32 trunk_f32 act16 act4096 > gpurun_out/r4f_grid.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4f_bench20.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r4f_bench10.log 2>&1 || exit $?
bash tools/prof_train.sh gpurun_out/r4f_c3prof
