set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench_train.py --steps 5 --warmup 2 > gpurun_out/tp_bench.log 2>&1 && \
timeout -k 10 300 python tools/torch_prof_train.py --host > gpurun_out/tp_host.log 2>&1 && \
timeout -k 10 300 python tools/torch_prof_train.py --syncs > gpurun_out/tp_syncs.log 2>&1
