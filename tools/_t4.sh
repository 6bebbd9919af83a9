cd ${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 -k "huffman or decode or cli" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; exit $rc
