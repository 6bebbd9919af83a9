#!/bin/bash
# Time the IE_PROFILE build with sections ablated (IE_ABLATE bits, see tools/gpu_pmc_ablate_insts.sh;
# 4096 = no pixel loads): us per 16-frame launch for each value in ABLATES.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
export IE_LIB=$R/imageencoder_amd/lib/var_prof/libie_hip.so
for ab in ${ABLATES:-0}; do
  echo -n "ablate=$ab "
  IE_ABLATE=$ab timeout -k 10 120 python tools/pmc_probe.py fast 16 2>&1 | grep mode
done
