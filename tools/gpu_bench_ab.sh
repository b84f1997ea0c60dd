# GPU run: order-balanced A/B of the default bench step vs --x3-kernel $V (no per-launch timers, no legs)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python bench.py --no-legs --no-cpu-baseline --steps 20 --no-op-timers > gpurun_out/bab_def_$i.log 2>&1 && \
timeout -k 10 200 python bench.py --no-legs --no-cpu-baseline --steps 20 --no-op-timers --x3-kernel $V > gpurun_out/bab_v_$i.log 2>&1 || exit 1
done
