#!/bin/bash
# GPU tests on the product build (TESTS, default: the encoder's parity tests), then an in-process
# A/B of the variant libraries named in AB (imageencoder_amd/lib/var_NAME; "product": the in-tree build).
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
TESTS=${TESTS:-tests/test_gpu_encode.py}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
libs=""; for v in $AB; do
  if [ "$v" = product ]; then libs="$libs imageencoder_amd/lib/libie_hip.so"; else libs="$libs imageencoder_amd/lib/var_$v/libie_hip.so"; fi
done
timeout -k 10 300 python tools/ab.py --rounds ${ROUNDS:-9} $ABARGS $libs 2>&1 | tail -12
