# round 4: bench after the GC fix, host-side profile of the C3 step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4h_bench.log 2>&1 || exit $?
timeout -k 10 240 python3 tools/host_profile.py --steps 5 > gpurun_out/r4h_hostprof.log 2>&1
