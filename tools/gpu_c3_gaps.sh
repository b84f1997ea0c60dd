# C3 host-side state: device allocations after the bench's own 4 warm-up steps, the bench_train line (timed 10 steps),
# and the idle gaps of 2 steps attributed to host frames (tools/gap_attrib.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/alloc_probe.py --steps 6 --warmup 4 > gpurun_out/c3g_alloc.log 2>&1 || exit $?
timeout -k 10 300 python3 bench_train.py > gpurun_out/c3g_bench.log 2>&1 || exit $?
timeout -k 10 300 python3 tools/gap_attrib.py --steps 2 --min-us 40 --out gpurun_out/c3g_gaps.txt > gpurun_out/c3g_gap.log 2>&1 || exit $?
