# C5 state at HEAD: rocprofv3 kernel trace of bench_zopt.py (KernelGAN kernel), last 4 iterations summarised
set -o pipefail
mkdir -p gpurun_out
bash tools/prof_zopt.sh gpurun_out/c5s || exit $?
python3 tools/trace_window.py gpurun_out/c5s/trace/run_kernel_trace.csv -360 4 > gpurun_out/c5s_kernels.md || exit $?
