#!/bin/bash
# Decode timing over environment settings: CONFIGS="VAR=V,VAR=V ..." (one config per word),
# tools/prof_decode.py for 4x4 (and 8x8 with N8=1).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
for cfg in $CONFIGS; do
  envs=$(echo $cfg | tr ',' ' ')
  env $envs timeout -k 10 120 python3 tools/prof_decode.py 4 ${KINDS:-U,M,flat} 2>&1 | grep -v amdgpu.ids | sed "s/^/$cfg /" || exit 1
  if [ -n "$N8" ]; then env $envs timeout -k 10 120 python3 tools/prof_decode.py 8 U,flat 2>&1 | grep -v amdgpu.ids | sed "s/^/$cfg /" || exit 1; fi
done
