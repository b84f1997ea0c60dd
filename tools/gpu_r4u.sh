# round 4: fused HR convs, stencil-sum kernel v2: its parity tests, the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "fused or c2_production or full_size or golden" > gpurun_out/r4u_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4u_bench.log 2>&1 || exit $?
