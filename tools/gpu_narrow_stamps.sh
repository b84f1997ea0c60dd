# Stamped 12-column x3 conv at config-2 / config-5 widths: per-workgroup durations of the last (partial) column strip
# against the others, on the previous ablation library (exp_lib/libesr_exphead.so) and the current one.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/narrow_stamps.log
: > $out
for lib in exphead exp; do
  echo "== $lib" >> $out
  ESR_AMD_LIB=$PWD/exp_lib/libesr_$lib.so timeout -k 10 120 python3 tools/x3c_stamps.py 16:148:128:148 16:148:128:144 16:172:128:172 >> $out 2>&1 || exit $?
done
