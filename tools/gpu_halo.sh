# halo-tile discriminator kernel: op tests vs float64, determinism bisection, A/B timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_disc.py -x -q --timeout 200 --timeout-method thread -p no:warnings > gpurun_out/halo_tests.log 2>&1 || exit $?
bash tools/gpu_det.sh || exit $?
timeout -k 10 300 python -u tools/dconv_ab.py > gpurun_out/halo_ab.log 2>&1
