# Record-decode GPU tests, then decode timings per content kind for 4x4 and 8x8
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_files.py tests/test_gop.py -m gpu -x -q --timeout 120 --timeout-method thread -k "decode or gop" > $O/pytest_dec.log 2>&1
rc=$?; tail -3 $O/pytest_dec.log; [ $rc -eq 0 ] || exit $rc
IE_HDR_BITS=165 timeout -k 10 120 python3 tools/prof_decode.py 4 ${K4:-G,U,M,ex4} || exit 1
IE_HDR_BITS=549 timeout -k 10 120 python3 tools/prof_decode.py 8 ${K8:-G,U,M,ex1} || exit 1
