#!/bin/bash
# NOTE: stamps/ablations need an IE_PROFILE build: tools/variants.sh prof "-DIE_PROFILE=1", then IE_LIB=imageencoder_amd/lib/var_prof/libie_hip.so
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out; mkdir -p $O; cd $R
for ab in ${ABS:-0}; do
IE_ABLATE=$ab IE_STAMPS=$O/stamps_ab$ab.bin timeout -k 10 300 python3 tools/pmc_probe.py fast 16 > $O/stamps_ab$ab.log 2>&1
rc=$?; echo "probe ab$ab rc=$rc"; cat $O/stamps_ab$ab.log; [ $rc -eq 0 ] || exit $rc
python3 tools/stamps.py $O/stamps_ab$ab.bin
done
