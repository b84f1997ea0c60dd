# GPU run: every -m gpu test (no -x), smoke(), the default bench, a rocprofv3 kernel trace of the C3 step, then the
# C5 split-precision grid check and the training-loop margins
set -o pipefail
tag=${1:-r3b}
mkdir -p gpurun_out
timeout -k 10 780 python -u -m pytest tests -m gpu -v -rs --timeout 300 --timeout-method thread -p no:warnings > gpurun_out/${tag}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 && \
timeout -k 10 240 python bench.py > gpurun_out/${tag}_bench.log 2>&1 && \
bash tools/prof_train.sh gpurun_out/${tag}_c3prof && \
python tools/trace_window.py gpurun_out/${tag}_c3prof/trace/run_kernel_trace.csv -560 3 > gpurun_out/${tag}_c3prof_kernels.txt 2>&1 && \
python tools/trace_gaps.py gpurun_out/${tag}_c3prof/trace/run_kernel_trace.csv 560 25 > gpurun_out/${tag}_c3prof_gaps.txt 2>&1 && \
ESR_DGRAD_X3=0 timeout -k 10 200 python -u tools/diag_grid.py c5:x3 > gpurun_out/${tag}_c5_fwdx3_bwdf32.log 2>&1 && \
timeout -k 10 400 python -u tools/loop_margin.py x3:x3 x3:x6 f32:f32 > gpurun_out/${tag}_margins.log 2>&1
rc=$?
rm -f gpurun_out/${tag}_c3prof/trace/*.csv.gz 2>/dev/null
exit $rc
