#!/bin/bash
# Stall attribution of the config-2 NTT kernels (scripts/prof_ntt.py), one SQ
# counter group per rocprofv3 pass.   RUN=name bash scripts/gpu_stall_ntt.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-stall_ntt}
mkdir -p $OUT
B="python scripts/prof_ntt.py ${POLYS:-256}"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_WAVES SQ_LEVEL_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/p$i -o p$i --output-format csv -- $B > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python scripts/stall_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
