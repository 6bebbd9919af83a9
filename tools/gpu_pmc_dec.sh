#!/bin/bash
# Instruction mix and utilisation counters of the record-decode kernels (tools/prof_decode.py, one
# 4K frame of content KIND, N x N), one rocprofv3 --pmc pass per counter set, each under its own
# time limit.  -> gpurun_out/pmcdec/summary.txt
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmcdec; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
N=${N:-4}; KIND=${KIND:-U}
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p$N$i -o run -- python3 $R/tools/prof_decode.py $N $KIND > $O/p$N$i.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; tail -3 $O/p$N$i.log; exit $rc; fi
  python3 $R/tools/pmc_summary.py $(find $O/p$N$i -name "*counter_collection.csv") | grep "rec_\|compose" >> $O/summary.txt
done
cat $O/summary.txt
