#!/bin/bash
# One GPU session running a selection of -m gpu tests: tools/gpu_tests.sh <pytest args...>
# (the GPU step has its own limit; its log lands in gpurun_out/pytest_sel.log)
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread "$@" > $O/pytest_sel.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" $O/pytest_sel.log | tail -3
exit $rc
