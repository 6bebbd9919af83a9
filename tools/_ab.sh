cd ${GRAFT_REPO_ROOT:-/root/repo}
export WL=${WL:-c2}
bash tools/gpu_variants.sh
IE_LIB= timeout -k 10 300 python bench.py --workload $WL --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_default.log 2>&1; echo "default rc=$?"; tail -1 gpurun_out/bench_default.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['launch_us'], d['roofline']['frac'], d['fallback_coefs_per_launch'])"
