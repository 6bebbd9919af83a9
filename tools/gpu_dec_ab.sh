#!/bin/bash
# Decode A/B: the exact-parse tests (unless TESTS=none), then tools/prof_decode.py over table-wave
# geometries (CONFIGS: "tm:hbits ...") for 4x4 (and 8x8 with N8=1).
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
if [ "${TESTS:-x}" != "none" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_files.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/dec_tests.log 2>&1; rc=$?; tail -2 gpurun_out/dec_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for cfg in ${CONFIGS:-"1:11 2:11 2:12"}; do
  tm=${cfg%:*}; hb=${cfg#*:}
  IE_REC_TM=$tm IE_REC_HB=$hb timeout -k 10 120 python3 tools/prof_decode.py 4 ${KINDS:-U,M,flat} 2>&1 | grep -v amdgpu.ids | sed "s/^/tm=$tm hb=$hb /" || exit 1
  if [ -n "$N8" ]; then IE_REC_TM=$tm IE_REC_HB=$((hb+2)) timeout -k 10 120 python3 tools/prof_decode.py 8 U,flat 2>&1 | grep -v amdgpu.ids | sed "s/^/tm=$tm hb=$((hb+2)) /" || exit 1; fi
done
