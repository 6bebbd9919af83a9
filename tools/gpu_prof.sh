#!/bin/bash
# Stamps (IE_PROFILE build) + PMC instruction/wait mix of the product build, 16-frame 4K launches.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
IE_LIB=$R/imageencoder_amd/lib/var_prof/libie_hip.so IE_STAMPS=$O/stamps.bin timeout -k 10 300 python3 tools/pmc_probe.py fast 16 > $O/stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/stamps.py $O/stamps.bin 2.1 | head -16
bash tools/gpu_pmc.sh
