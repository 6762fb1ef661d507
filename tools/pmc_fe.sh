#!/bin/bash
# SQ counter passes over the FE kernel alone (tools/fe_bench pmc): one pass per
# counter group (rocprofv3 does not split groups over passes)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for g in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD" \
         "GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $g --output-format csv -d gpurun_out/pmc_fe$i -o run -- ${1:-./tools/fe_bench} pmc > gpurun_out/pmc_fe$i.log 2>&1 || exit $i
done
python tools/pmc_summary.py gpurun_out/pmc_fe1 gpurun_out/pmc_fe2 gpurun_out/pmc_fe3
