set -o pipefail
mkdir -p gpurun_out
export AB_ROUNDS=4 AB_REPS=20 ESR_AMD_LIB=$PWD/tools/exp/libesr_exp.so
AB_COUT=64 AB_CIN=192 AB_HW=148 AB_VARIANTS=50,51,52,53,54 AB_DIAG=51,52,53,54 timeout -k 10 300 python tools/x3_ab.py > gpurun_out/ab3_n64.log 2>&1 && \
AB_COUT=32 AB_CIN=128 AB_HW=148 AB_VARIANTS=50,51,52,53,54 AB_DIAG=51,52,53,54 timeout -k 10 300 python tools/x3_ab.py > gpurun_out/ab3_n32.log 2>&1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export AB_ROUNDS=1 AB_REPS=5 AB_COUT=64 AB_CIN=192 AB_HW=148 AB_VARIANTS=1,50
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc3/p1 -o run -- python3 $R/tools/x3_ab.py > $R/gpurun_out/pmc3_p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc3/p2 -o run -- python3 $R/tools/x3_ab.py > $R/gpurun_out/pmc3_p2.log 2>&1
