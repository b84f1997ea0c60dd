# C3 state at HEAD: rocprofv3 kernel trace of bench_train.py (3 timed steps) summarised over the last 3 steps, and the
# device allocations made after warm-up (tools/alloc_probe.py).
set -o pipefail
mkdir -p gpurun_out
bash tools/prof_train.sh gpurun_out/c3s || exit $?
python3 tools/trace_window.py gpurun_out/c3s/trace/run_kernel_trace.csv -400 3 > gpurun_out/c3s_kernels.md || exit $?
timeout -k 10 300 python3 tools/alloc_probe.py --steps 4 --warmup 6 > gpurun_out/c3s_alloc.log 2>&1 || exit $?
rm -rf gpurun_out/c3s/trace/*.csv.gz
