#!/bin/bash
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out; mkdir -p $O; cd $R
for ab in ${ABS:-0}; do
IE_ABLATE=$ab IE_STAMPS=$O/stamps_ab$ab.bin timeout -k 10 300 python3 tools/pmc_probe.py fast 16 > $O/stamps_ab$ab.log 2>&1
rc=$?; echo "probe ab$ab rc=$rc"; cat $O/stamps_ab$ab.log; [ $rc -eq 0 ] || exit $rc
python3 tools/stamps.py $O/stamps_ab$ab.bin
done
