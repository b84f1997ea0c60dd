# GPU run: all -m gpu tests, smoke(), the default bench line, then the rocprofv3 kernel-trace + PMC passes of the
# default bench summarised into gpurun_out/prof/summary (tools/prof_summary.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:warnings > gpurun_out/final_tests.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/final_bench.log 2>&1 && \
bash tools/prof_bench.sh gpurun_out/prof --no-legs && \
python3 tools/prof_summary.py gpurun_out/prof gpurun_out/prof/summary > gpurun_out/final_prof.log 2>&1
