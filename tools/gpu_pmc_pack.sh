#!/bin/bash
# Counters of the C5 Huffman pack (tools/c5_breakdown.py drives encode + Huffman batches): two
# rocprofv3 --pmc passes (instruction mix; waits, LDS bank conflicts), pack / first-scan kernels.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmcp; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
p=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  p=$((p+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/p$p -o run -- python3 $R/tools/c5_breakdown.py > $O/p$p.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "pass $p rc=$rc"; tail -3 $O/p$p.log; exit $rc; fi
  python3 $R/tools/pmc_summary.py $(find $O/p$p -name "*counter_collection.csv") | grep -E "pack_kernel|first_scan|encode4p"
done
