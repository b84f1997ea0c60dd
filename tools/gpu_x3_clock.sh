# GPU run: PMC pass over tools/x3_ab.py (default kernel, one shape per run): GRBM_GUI_ACTIVE (GPU cycles at the actual
# clock), SQ_BUSY_CYCLES, SQ_VALU_MFMA_BUSY_CYCLES, SQ_WAVE_CYCLES, with the kernel trace for the durations
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/clk
cd /tmp && export TMPDIR=/tmp
export AB_VARIANTS=1 AB_ROUNDS=1 AB_REPS=5
AB_CIN=128 AB_COUT=32 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/clk/n32 -o run -- python3 $R/tools/x3_ab.py > $R/gpurun_out/clk/n32.log 2>&1 && \
AB_CIN=192 AB_COUT=64 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/clk/n64 -o run -- python3 $R/tools/x3_ab.py > $R/gpurun_out/clk/n64.log 2>&1
