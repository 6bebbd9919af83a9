#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
rc2=$?
echo "bench rc=$rc2"
tail -5 gpurun_out/bench.log
exit $rc2
