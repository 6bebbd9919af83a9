R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_files.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pipelined" 2>&1 | tail -2 || exit 1
for opt in "" "--no-pack-overlap" ""; do
timeout -k 10 300 python3 bench.py --workload c5 --steps 10 --warmup 2 --no-cpu --no-e2e --no-decode --no-gop --no-single-frame $opt > gpurun_out/c5x.json 2>gpurun_out/c5x.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/c5x.json')); print('$opt', d['value'], d['ms_per_step'], d['check']['bit_exact'])"
done
bash tools/gpu_c5trace.sh | tail -3
