# esr_axpby_gs: the row-walking kernel (knob 1, product) vs 4 items in flight per thread (knob 2) on the C5 and C3
# steps (ablation library, tools/knob_bench.py), order-balanced
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/axpby_ab.log
: > $out
export ESR_AMD_LIB=exp_lib/libesr_exp.so
for v in 1 2 1 2; do
  echo "== axpby_rows=$v C5" >> $out
  timeout -k 10 200 python3 tools/knob_bench.py axpby_set_rows=$v -- bench_zopt.py --steps 10 2>/dev/null | grep '^{' >> $out || exit $?
  echo "== axpby_rows=$v C3" >> $out
  timeout -k 10 200 python3 tools/knob_bench.py axpby_set_rows=$v -- bench_train.py --steps 8 2>/dev/null | grep '^{' >> $out || exit $?
done
