#!/bin/bash
# GPU tests on the product build, then an in-process A/B of the listed variant libraries.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
libs=""; for v in $AB; do libs="$libs imageencoder_amd/lib/var_$v/libie_hip.so"; done
timeout -k 10 300 python tools/ab.py --rounds 9 $libs 2>&1 | tail -8
