# config-3 training step and config-5 Z iteration: timings (deferred overflow checks on/off), a kernel trace of C3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench_train.py --steps 5 --warmup 4 > gpurun_out/c3_default.log 2>&1 || exit $?
ESR_DEFER_OVERFLOW=0 timeout -k 10 300 python -u bench_train.py --steps 5 --warmup 4 > gpurun_out/c3_eager.log 2>&1 || exit $?
timeout -k 10 300 python -u bench_zopt.py --steps 5 --warmup 2 > gpurun_out/c5_default.log 2>&1 || exit $?
bash tools/prof_train.sh gpurun_out/c3prof || exit $?
python tools/trace_window.py gpurun_out/c3prof/trace/run_kernel_trace.csv -600 3 > gpurun_out/c3prof_kernels.txt 2>&1
python tools/trace_gaps.py gpurun_out/c3prof/trace/run_kernel_trace.csv 600 25 > gpurun_out/c3prof_gaps.txt 2>&1
rm -rf gpurun_out/c3prof/trace/*.csv.gz 2>/dev/null; true
