# rocprofv3 SQ-counter passes (each its own run, <= 8 SQ / 2 GRBM counters) over the default inference bench at HEAD
# (product library, 2 timed steps): usage bash tools/pmc_bench_sq.sh OUTDIR ; summarise with
# python3 tools/pmc_x3_summary.py OUTDIR (per x3 conv instantiation: conv_x3c_kernel<...> and its LDS size)
out=$1
R=$GRAFT_REPO_ROOT; mkdir -p $R/$out
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM" \
           "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $R/$out/p$i -o run -- python3 $R/bench.py --no-legs --no-cpu-baseline --steps 2 --warmup 1 > $R/$out/p$i.log 2>&1 || exit $?
done
