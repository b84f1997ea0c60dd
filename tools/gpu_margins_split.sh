# Which part of the x3 generator step carries the training-loop drift: G x3 forward with D f32, and the x3 backward
# halves switched to exact fp32 one at a time (ESR_WGRAD_X3 / ESR_DGRAD_X3)
set -o pipefail
mkdir -p gpurun_out
for cfg in "1 1" "0 1" "1 0" "0 0"; do
  set -- $cfg
  echo "== ESR_WGRAD_X3=$1 ESR_DGRAD_X3=$2" >> gpurun_out/margins_split.log
  ESR_WGRAD_X3=$1 ESR_DGRAD_X3=$2 timeout -k 10 300 python -u tools/loop_margin.py x3:f32 >> gpurun_out/margins_split.log 2>&1 || exit $?
done
