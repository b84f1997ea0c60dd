# GPU run: rocprofv3 kernel trace + FETCH/WRITE PMC passes of the default bench, summarised (tools/prof_summary.py)
set -o pipefail
mkdir -p gpurun_out
bash tools/prof_bench.sh gpurun_out/prof --no-legs && \
python3 tools/prof_summary.py gpurun_out/prof gpurun_out/prof/summary > gpurun_out/prof_summary.log 2>&1
