# GPU run: rocprofv3 kernel trace of bench_train.py (config 3), per-kernel window summary and idle gaps
set -o pipefail
mkdir -p gpurun_out
bash tools/prof_train.sh gpurun_out/tp2 && \
T=$(ls gpurun_out/tp2/trace/*kernel_trace.csv | head -1) && \
python3 tools/trace_window.py $T -560 3 > gpurun_out/tp2_window.txt 2>&1 && \
python3 tools/trace_gaps.py $T 560 25 > gpurun_out/tp2_gaps.txt 2>&1
