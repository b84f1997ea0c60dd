# A/B of the multi-stream inference forward (engine.STREAMS: the config-2 batch in S parts on S HIP streams), bench.py
# headline only, no per-launch timers (pure throughput); order S = 1 2 3 4 1 2; then the batch/parity tests that run
# the split path (B = 32 production grid vs the oracle and bitwise vs B = 1; batch invariance; overflow fallback)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/${1:-streams}_ab.log
: > $out
for s in 1 2 3 4 1 2; do
  echo "== ESR_STREAMS=$s" >> $out
  ESR_STREAMS=$s timeout -k 10 200 python3 bench.py --no-legs --no-cpu-baseline --no-op-timers --steps 20 --warmup 5 2>/dev/null | grep '^{' >> $out || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "production_grid or batch_invariance or overflow or full_size or fused_equals" >> $out 2>&1 || exit $?
