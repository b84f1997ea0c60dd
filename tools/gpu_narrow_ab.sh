# Narrow last column tile of the x3 conv: parity tests of the touched kernels, the width probe, then config-2 / config-5
# steps on the new library against the previous one (exp_lib/libesr_head.so, built from the parent commit), order A B A B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "ring_kernel or n64_explicit or upconv2x_phases_x3 or conv3x3_layer_x3 or c2_production or full_size or multistream or xcd_tile or nsplit" \
  > gpurun_out/narrow_tests.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/x3_width_probe.py 16 148 128 144,148,156 > gpurun_out/narrow_probe.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/x3_width_probe.py 16 172 128 168,172,180 >> gpurun_out/narrow_probe.log 2>&1 || exit $?
out=gpurun_out/narrow_ab.log
: > $out
for r in 1 2; do
  for lib in head new; do
    echo "== C2 $lib" >> $out
    if [ $lib = head ]; then export ESR_AMD_LIB=$PWD/exp_lib/libesr_head.so; else unset ESR_AMD_LIB; fi
    timeout -k 10 300 python3 bench.py --no-legs --steps 20 --warmup 5 --no-op-timers --no-cpu-baseline 2>/dev/null | grep '^{' >> $out || exit $?
  done
done
for r in 1 2; do
  for lib in head new; do
    echo "== C5 $lib" >> $out
    if [ $lib = head ]; then export ESR_AMD_LIB=$PWD/exp_lib/libesr_head.so; else unset ESR_AMD_LIB; fi
    timeout -k 10 300 python3 bench_zopt.py --steps 10 2>/dev/null | grep '^{' >> $out || exit $?
  done
done
