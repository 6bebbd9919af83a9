#!/bin/bash
# profiling aid: time the 4x4 FAST encoder with sections disabled (outputs are wrong)
for ab in 0 1 2 4 8 16 7 15 31; do
  echo -n "ablate=$ab "
  IE_ABLATE=$ab timeout -k 10 120 python tools/pmc_probe.py fast 16 | grep mode
done
