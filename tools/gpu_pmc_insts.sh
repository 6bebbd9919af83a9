#!/bin/bash
# Dynamic instruction mix and stall counters of the C2 encode (tools/pmc_probe.py, 16 4K frames per
# launch): one rocprofv3 --pmc pass per counter set, each under its own time limit.  LIBS: libie_hip.so
# paths to compare (default: the in-tree product library).
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmci; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
LIBS=${LIBS:-$R/imageencoder_amd/lib/libie_hip.so}
li=0
for lib in $LIBS; do
  li=$((li+1)); i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT" \
             ${EXTRA_SETS}; do
    i=$((i+1))
    IE_LIB=$R/$lib timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/l${li}p$i -o run -- python3 $R/tools/pmc_probe.py fast 16 > $O/l${li}p$i.log 2>&1
    rc=$?; echo "lib $lib pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $O/l${li}p$i.log; exit $rc; fi
  done
  echo "== $lib" >> $O/summary.txt
  python3 $R/tools/pmc_summary.py $(find $O/l${li}p* -name "*counter_collection.csv") | grep encode >> $O/summary.txt
done
cat $O/summary.txt
exit 0
