#!/bin/bash
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmc2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1
grep -o "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_0-9]*\|SQ_WAIT[A-Z_0-9]*\|SQ_INST_LEVEL[A-Z_0-9]*\|SQ_LEVEL[A-Z_0-9]*\|TA_[A-Z_]*BUSY[A-Z_0-9]*\|TCP_[A-Z_]*STALL[A-Z_0-9]*" $O/counters.txt | sort -u | head -80
i=0
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" \
           "SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM SQ_ACCUM_PREV_HIRES SQ_WAVES SQ_BUSY_CU_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $R/tools/pmc_probe.py fast 16 > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $O/p$i.log; fi
done
python3 $R/tools/pmc_summary.py $(find $O -name "*counter_collection.csv") | grep encode_kernel
exit 0
