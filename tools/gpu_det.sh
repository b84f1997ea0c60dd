# determinism bisection of the training step (tools/loop_determinism.py) over the D kernels
set -o pipefail
mkdir -p gpurun_out
for env in "ESR_DCONV_HALO=1 ESR_FUSED_BN=1" "ESR_DCONV_HALO=0 ESR_FUSED_BN=1" "ESR_DCONV_HALO=1 ESR_FUSED_BN=0" "ESR_DCONV_HALO=0 ESR_FUSED_BN=0"; do
  echo "== $env" >> gpurun_out/det2.log
  env $env timeout -k 10 300 python -u tools/loop_determinism.py f32:f32 >> gpurun_out/det2.log 2>&1 || exit $?
done
