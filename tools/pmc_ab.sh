#!/bin/bash
# Two rocprofv3 --pmc passes (SQ stall / LDS counters) over tools/x3_ring_ab.py; env AB_* passes through.
# usage: tools/pmc_ab.sh OUTDIR
out=$1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; mkdir -p $R/$out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/$out/p1 -o run -- python3 $R/tools/x3_ring_ab.py > $R/$out/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT --output-format csv -d $R/$out/p2 -o run -- python3 $R/tools/x3_ring_ab.py > $R/$out/p2.log 2>&1 || exit $?
