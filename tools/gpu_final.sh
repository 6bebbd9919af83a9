#!/bin/bash
# Round-end GPU session: every -m gpu test, smoke, the default bench line, the C2 kernel trace.
# Each GPU step has its own limit; a fault / abort / timeout ends the script.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $O/bench_default.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-single-frame --no-e2e --no-decode --no-gop > $O/prof_stats.log 2>&1
rc=$?; echo "rocprof stats rc=$rc"; tail -1 $O/prof_stats.log
exit $rc
