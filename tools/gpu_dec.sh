# Decode GPU session: the decode tests (TESTS=none skips them), then decode timings per content kind
# (speculative parse with warm-up WARMS chunks, and the exact parse alone) for n in NS.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
if [ "${TESTS}" != "none" ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_files.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "decode" > $O/pytest_dec.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_dec.log; [ $rc -eq 0 ] || exit $rc
fi
for n in ${NS:-4 8}; do
  for wu in ${WARMS:-1}; do IE_DEC_WARM=$wu timeout -k 10 120 python tools/prof_decode.py $n $KINDS || exit 1; echo "(warm $wu)"; done
  IE_DEC_SPEC=0 timeout -k 10 120 python tools/prof_decode.py $n $KINDS || exit 1; echo "(exact)"
done
