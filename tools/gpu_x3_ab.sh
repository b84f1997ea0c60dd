# GPU run: x3 conv A/B (tools/x3_ab.py) of the variants in $AB_VARIANTS at N=32 (148^2 and 96^2) and N=64 (148^2)
set -o pipefail
mkdir -p gpurun_out
export AB_ROUNDS=${AB_ROUNDS:-4} AB_REPS=${AB_REPS:-20}
AB_HW=148,96 timeout -k 10 300 python tools/x3_ab.py > gpurun_out/x3ab_n32.log 2>&1 && \
AB_COUT=64 timeout -k 10 240 python tools/x3_ab.py > gpurun_out/x3ab_n64.log 2>&1
