#!/bin/bash
# P-frame session: the gop tests, then the P-frame timing (tools/prof_gop.py) and its kernel trace.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/pf; mkdir -p $O; cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gop.py tests/test_gpu_files.py tests/test_gpu_stream.py tests/test_gpu_encode.py tests/test_integration.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/prof_gop.py > $O/gop.log 2>&1 || { tail -5 $O/gop.log; exit 1; }
grep -v amdgpu.ids $O/gop.log | tail -6
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 $R/tools/prof_gop.py > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/pf/tr/run_kernel_stats.csv")):
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.2f} us")
PY
