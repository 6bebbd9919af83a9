#!/bin/bash
# Dynamic VALU / SALU / LDS instruction counts (one rocprofv3 --pmc pass each) of the C2 encode for
# every library in LIBS: phase costs from ablation builds (IE_P_ABL) by difference.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmcv; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
li=0
for lib in $LIBS; do
  li=$((li+1))
  IE_LIB=$R/$lib timeout -s KILL 90 rocprofv3 --pmc ${COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES} --kernel-trace --output-format csv -d $O/l$li -o run -- python3 $R/tools/pmc_probe.py fast 16 > $O/l$li.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "lib $lib rc=$rc"; tail -3 $O/l$li.log; exit $rc; fi
  echo "== $lib"
  python3 $R/tools/pmc_summary.py $(find $O/l$li -name "*counter_collection.csv") | grep "encode4"
done
