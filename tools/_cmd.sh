cd ${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_c5.log 2>&1; rc=$?; tail -1 gpurun_out/bench_c5.log; exit $rc
