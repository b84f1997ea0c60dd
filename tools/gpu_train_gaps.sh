# GPU run: rocprofv3 kernel trace of bench_train.py (config 3) and its largest idle gaps
set -o pipefail
mkdir -p gpurun_out
bash tools/prof_train.sh gpurun_out/tg && \
python3 tools/trace_gaps.py $(ls gpurun_out/tg/trace/*kernel_trace.csv | head -1) 580 40 > gpurun_out/tg_gaps.txt 2>&1
