# loop margins on the regenerated fixtures (reference ensemble), all precision pairs; 3-run determinism
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/loop_determinism.py f32:f32 > gpurun_out/det5.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/loop_margin.py x3:x3 x3:x6 x3:f32 f32:f32 f32:x3 > gpurun_out/margins2.log 2>&1
