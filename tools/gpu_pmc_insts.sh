#!/bin/bash
# Dynamic instruction mix and stall counters of the C2 encode (tools/pmc_probe.py, 16 4K frames per
# launch): one rocprofv3 --pmc pass per counter set, each under its own time limit.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmci; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT" \
           ${EXTRA_SETS}; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $R/tools/pmc_probe.py fast 16 > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $O/p$i.log; exit $rc; fi
done
python3 $R/tools/pmc_summary.py $(find $O -name "*counter_collection.csv") | grep encode_kernel > $O/summary.txt
cat $O/summary.txt
exit 0
