#!/bin/bash
# Round-2 GPU session A: GPU tests, default bench (c2), c4 at one GPU, a two-rank rehearsal of the
# multi-GPU bench (gloo, both ranks on the one GPU), each step under its own time limit.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
fatal() { local rc=$1; [ $rc -ge 124 ] || [ $rc -lt 0 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; }
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log; fatal $rc && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-e2e --no-decode > $O/bench_c2.log 2>&1
rc=$?; echo "bench c2 rc=$rc"; tail -1 $O/bench_c2.log; fatal $rc && exit $rc
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 2 > $O/bench_c4.log 2>&1
rc=$?; echo "bench c4 rc=$rc"; tail -1 $O/bench_c4.log; fatal $rc && exit $rc
IE_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 > $O/bench_g2.log 2>&1
rc=$?; echo "bench gloo x2 rc=$rc"; tail -3 $O/bench_g2.log
exit 0
