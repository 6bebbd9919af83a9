cd ${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/c5_breakdown.py 2>&1 | grep -v amdgpu.ids
for L in imageencoder_amd/lib/var_0head/libie_hip.so imageencoder_amd/lib/libie_hip.so; do
IE_LIB=$L timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu > gpurun_out/b5.log 2>&1; echo "$L rc=$?"; tail -1 gpurun_out/b5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['launch_us'])"
done
