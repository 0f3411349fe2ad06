#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each, per the microarch guide's
# per-block limits) over the C5 in-batch CE forward+backward
# (tools/microbench_inbatch.py --c5): per-kernel averages into
# gpurun_out/$TAG/inbatch_pmc.txt, for the VALU-vs-MFMA attribution of the
# LSE / ROW / COL passes of csrc/inbatch16.hip.
TAG=${1:-inbatch_pmc}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG; mkdir -p $O
P=/tmp/$TAG; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_LDS"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
  "SQ_VALU_MFMA_COEXEC_CYCLES"
)
i=0
for C in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d $P/p$i -o p -- python3 $R/tools/microbench_inbatch.py --c5 > $P/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i ($C) rc=$rc"; tail -3 $P/p$i.log; fi
  if [ $rc -eq 137 ] || [ $rc -eq 124 ]; then exit 1; fi
done
python3 $R/tools/pmc_dump.py $(find $P -name "*.db") --filter ib16 > $O/inbatch_pmc.txt
cat $O/inbatch_pmc.txt
