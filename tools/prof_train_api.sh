#!/bin/bash
# rocprofv3 kernel + HIP API trace of bench_train.py (config 3) -> OUTDIR/trace: which host calls the GPU's idle gaps
# follow (round-4 gap attribution; tools/gap_attrib.py is the torch.profiler form)
out=$1; shift
R=$GRAFT_REPO_ROOT; mkdir -p $R/$out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d $R/$out/trace -o run -- python3 $R/bench_train.py --steps 3 --warmup 5 "$@" > $R/$out/trace.log 2>&1
