#!/bin/bash
# Encoder tests, then the C2 bench line under environment settings (CONFIGS: "VAR=V,VAR=V ..."; the
# first word "default"): small-launch geometry A/B.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
if [ "${TESTS:-x}" != "none" ]; then bash tools/gpu_tests.sh ${TESTARGS:-tests/test_gpu_encode.py tests/test_gpu_files.py -x -q} || exit 1; fi
i=0
for cfg in ${CONFIGS:-default IE_SMALL_TILES=0}; do
  envs=$(echo $cfg | tr ',' ' '); [ "$cfg" = default ] && envs=""
  env $envs timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-decode --no-gop ${BARGS} > $O/bench_s$i.log 2>&1 || { tail -5 $O/bench_s$i.log; exit 1; }
  python3 -c "
import json, sys; d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'ms/step', d['ms_per_step'], 'launch_us', d['roofline']['launch_us'], 'single', d['single_frame'])" $O/bench_s$i.log $cfg
  i=$((i+1))
done
