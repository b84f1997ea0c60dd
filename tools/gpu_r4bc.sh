# round 4 final verification at HEAD: every GPU test, smoke(), the bench line, then the rocprofv3 passes over the
# default inference bench (kernel trace + stats; FETCH_SIZE; WRITE_SIZE), summarised on the box (the raw traces
# exceed what gpurun copies back)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4bc_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4bc_smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/r4bc_bench.log 2>&1 || exit $?
bash tools/prof_bench.sh gpurun_out/r4bc_prof || exit $?
python3 tools/prof_summary.py gpurun_out/r4bc_prof gpurun_out/r4bc_c2 > gpurun_out/r4bc_summary.log 2>&1 || exit $?
cp gpurun_out/r4bc_prof/trace/run_kernel_stats.csv gpurun_out/r4bc_c2_rocprof_kernel_stats.csv
rm -rf gpurun_out/r4bc_prof
