#!/bin/bash
# Dynamic instruction counts per ablation (SQ_INSTS_*), one rocprofv3 pass per ablation value.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmcab${TAG:+_$TAG}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for ab in ${ABLATES:-0 1 2 4 8 16}; do
  IE_ABLATE=$ab timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d $O/ab$ab -o run -- python3 $R/tools/pmc_probe.py fast 16 > $O/ab$ab.log 2>&1
  rc=$?; echo "ablate $ab rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/ab$ab.log; exit $rc; fi
  python3 $R/tools/pmc_summary.py $(find $O/ab$ab -name "*counter_collection.csv") | grep "encode_kernel" | grep -v meta | awk '{print $(NF-2), $NF}'
done
