# GPU run at HEAD: every -m gpu test (no -x, so every failure shows), smoke(), then the split-precision loop margins
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rs --timeout 300 --timeout-method thread -p no:warnings > gpurun_out/head_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/head_smoke.log 2>&1 && \
timeout -k 10 600 python -u tools/loop_margin.py > gpurun_out/head_margins.log 2>&1
