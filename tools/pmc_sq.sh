#!/bin/bash
# SQ counter passes over a program's kernels, one rocprofv3 --pmc run per
# counter group (rocprofv3 does not split groups over passes).
# usage: bash tools/pmc_sq.sh TAG PROGRAM [ARGS...]   -> gpurun_out/pmc_TAG{1,2,3}
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
i=0
for g in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAVES" \
         "GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $g --output-format csv -d gpurun_out/pmc_$tag$i -o run -- "$@" > gpurun_out/pmc_$tag$i.log 2>&1 || exit $i
done
python tools/pmc_summary.py gpurun_out/pmc_${tag}1 gpurun_out/pmc_${tag}2 gpurun_out/pmc_${tag}3
