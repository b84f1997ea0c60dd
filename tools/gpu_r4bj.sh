# round 4 final state: every GPU test (skip reasons listed), smoke(), the bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/r4bj_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4bj_smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/r4bj_bench.log 2>&1 || exit $?
