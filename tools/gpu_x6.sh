# x6 discriminator convolutions: op tests vs float64 (errors printed), D-step determinism, A/B timing, loop margins
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_disc.py -x -v -s --timeout 200 --timeout-method thread -p no:warnings -k "dconv_ops" > gpurun_out/x6_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u -m pytest tests/test_gpu_cem_adjoint.py -x -q --timeout 100 --timeout-method thread -p no:warnings > gpurun_out/adj_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/d_determinism.py > gpurun_out/ddet.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/dconv_ab.py > gpurun_out/x6_ab.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/loop_margin.py x3:x6 f32:x6 > gpurun_out/x6_margins.log 2>&1
