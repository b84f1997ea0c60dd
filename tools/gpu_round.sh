# GPU run at HEAD: every -m gpu test (no -x, every failure shows), smoke(), the default bench
# (usage: gpurun --timeout 1200 -- bash tools/gpu_round.sh TAG)
set -o pipefail
tag=${1:-head}
mkdir -p gpurun_out
timeout -k 10 780 python -u -m pytest tests -m gpu -v -rs --timeout 300 --timeout-method thread -p no:warnings > gpurun_out/${tag}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/${tag}_bench.log 2>&1
