# round 4: host run-ahead on this ROCm stack, eager vs graph, with memset / memcpy nodes
set -o pipefail
mkdir -p gpurun_out
P="python3 tools/graph_launch_probe.py 400 1200"
PROBE_MODE=memset timeout -k 10 120 $P > gpurun_out/r4o_memset.log 2>&1 || exit $?
PROBE_MODE=memcpy timeout -k 10 120 $P > gpurun_out/r4o_memcpy.log 2>&1 || exit $?
PROBE_MODE=memcpy DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 $P > gpurun_out/r4o_memcpy_nocap.log 2>&1 || exit $?
