#!/bin/bash
# NOTE: stamps/ablations need an IE_PROFILE build: tools/variants.sh prof "-DIE_PROFILE=1", then IE_LIB=imageencoder_amd/lib/var_prof/libie_hip.so
# profiling aid: time the 4x4 FAST encoder with sections disabled (outputs are wrong)
for ab in 0 1 2 4 8 16 7 15 31; do
  echo -n "ablate=$ab "
  IE_ABLATE=$ab timeout -k 10 120 python tools/pmc_probe.py fast 16 | grep mode
done
