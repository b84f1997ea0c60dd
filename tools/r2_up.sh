set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python bench.py --no-legs --no-cpu-baseline --steps 20 > gpurun_out/r2_up_v1_$i.log 2>&1 && \
timeout -k 10 200 python bench.py --no-legs --no-cpu-baseline --steps 20 --x3-kernel 63 > gpurun_out/r2_up_v63_$i.log 2>&1 || exit 1
done
