cd ${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab.py imageencoder_amd/lib/libie_hip.so 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python tools/ab.py --n 8 imageencoder_amd/lib/libie_hip.so 2>&1 | grep -v amdgpu.ids
