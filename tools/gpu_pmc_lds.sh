#!/bin/bash
# LDS pressure of the encode kernel (current library): bank-conflict cycles vs LDS-active cycles.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmclds; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
IE_N=${IE_N:-4} timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d $O -o run -- python3 $R/tools/pmc_probe.py fast 16 > $O/p.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/p.log; exit $rc; }
python3 $R/tools/pmc_summary.py $(find $O -name "*counter_collection.csv") | grep "encode_kernel" | grep -v meta
