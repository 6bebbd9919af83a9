#!/bin/bash
# PMC passes over tools/prof_decode.py (args: n kinds), summary of the record-parse kernels.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmcdec; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_INSTS_FLAT"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $R/tools/prof_decode.py "$@" > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/p$i.log; exit $rc; fi
done
python3 $R/tools/pmc_summary.py $(find $O -name "*counter_collection.csv") | grep "rec_"
