set -e
mkdir -p gpurun_out/pmc
R=$GRAFT_REPO_ROOT; P=/tmp/pmc; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
for K in 1 100; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -d $P/a$K -o a -- python3 $R/tools/prof_topk.py $K 1 > $P/a$K.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $P/b$K -o b -- python3 $R/tools/prof_topk.py $K 1 > $P/b$K.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INST_LEVEL_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_BRANCH -d $P/c$K -o c -- python3 $R/tools/prof_topk.py $K 1 > $P/c$K.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $P/f$K -o f -- python3 $R/tools/prof_topk.py $K 1 > $P/f$K.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum -d $P/w$K -o w -- python3 $R/tools/prof_topk.py $K 1 > $P/w$K.log 2>&1
python3 $R/tools/pmc_dump.py $(find $P -path "*[abcfw]$K/*" -name "*.db") --filter topk > $R/gpurun_out/pmc/k$K.txt
done
cat $R/gpurun_out/pmc/k*.txt
