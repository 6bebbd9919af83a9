cd ${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
ABARGS="--rounds 5 --n 8" bash tools/_ab2.sh && ABARGS="--rounds 5" bash tools/_ab2.sh
