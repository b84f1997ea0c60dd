# round 4 final verification at HEAD: every GPU test, smoke(), the bench line, then the rocprofv3 passes over the
# default inference bench (kernel trace + stats; FETCH_SIZE; WRITE_SIZE) for profiles/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4bb_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4bb_smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/r4bb_bench.log 2>&1 || exit $?
bash tools/prof_bench.sh gpurun_out/r4bb_prof
