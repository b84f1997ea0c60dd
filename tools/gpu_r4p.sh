# round 4: config-3 step with the training graphs off / HIP graph packet capture off (host run-ahead)
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_ab_env.sh ESR_TRAIN_GRAPHS 1 0 || exit $?
bash tools/gpu_ab_env.sh DEBUG_CLR_GRAPH_PACKET_CAPTURE 1 0 || exit $?
