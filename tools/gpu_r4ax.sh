# round 4 verification at HEAD: every GPU test, smoke(), the bench line, a torch.profiler view of the config-3 step,
# then a same-box A/B of the D bias-gradient column sums (ESR_DCONV_COLSUM 0 vs 1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4ax_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4ax_smoke.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py > gpurun_out/r4ax_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/torch_prof_train.py --device > gpurun_out/r4ax_torchdev.log 2>&1 || exit $?
bash tools/gpu_ab_env.sh ESR_DCONV_COLSUM 0 1
