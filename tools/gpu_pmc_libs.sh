#!/bin/bash
# Instruction mix (SQ_INSTS_*) of the encode kernel for every variant library given in LIBS.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmclibs; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for lib in ${LIBS}; do
  n=$(basename $(dirname $lib))
  IE_LIB=$R/$lib timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-trace --output-format csv -d $O/$n -o run -- python3 $R/tools/pmc_probe.py fast 16 > $O/$n.log 2>&1
  rc=$?; echo "== $n rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/$n.log; exit $rc; fi
  python3 $R/tools/pmc_summary.py $(find $O/$n -name "*counter_collection.csv") | grep "encode_kernel" | grep -v meta | awk '{print $(NF-2), $NF}' | tr '\n' ' '; echo
done
