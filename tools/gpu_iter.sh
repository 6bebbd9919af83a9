#!/bin/bash
# One build -> measure iteration on the GPU box: the MFMA layout probe, the encoder's GPU parity
# tests (TESTS), the C2 bench line, and an in-process A/B of the product library against the
# variant libraries named in AB (imageencoder_amd/lib/var_NAME).
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
set -o pipefail
timeout -k 10 60 ./tools/probe/mfma_i8_probe > $O/probe.txt 2>&1; rc=$?; cat $O/probe.txt; [ $rc -eq 0 ] || exit $rc
TESTS=${TESTS:-tests/test_gpu_encode.py}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-decode --no-gop --no-e2e > $O/bench_c2.json 2> $O/bench_c2.err
  rc=$?; echo "bench rc=$rc"; python -c "import json;d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ('value','ms_per_step','bit_exact')}, d['roofline']['launch_us'], d['roofline']['frac'], d.get('single_frame'))" || exit 1
fi
if [ -n "$AB" ]; then
  libs="imageencoder_amd/lib/libie_hip.so"; for v in $AB; do libs="$libs imageencoder_amd/lib/var_$v/libie_hip.so"; done
  timeout -k 10 300 python tools/ab.py --rounds ${ROUNDS:-7} $ABARGS $libs > $O/ab.log 2>&1; rc=$?
  grep -v "^running" $O/ab.log | tail -12; [ $rc -eq 0 ] || { grep "^running" $O/ab.log | tail -1; exit $rc; }
fi
