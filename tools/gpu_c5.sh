( while sleep 50; do echo "[hb $(date +%T)]"; done ) &
HB=$!
trap 'kill $HB' EXIT
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_files.py -m gpu -x -q --timeout 120 --timeout-method thread -k "counted or huffman" 2>&1 | tail -3 || exit 1
timeout -k 10 300 python3 bench.py --workload c5 --steps 10 --warmup 2 --no-cpu --no-e2e --no-decode --no-gop > gpurun_out/c5.json 2>gpurun_out/c5.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/c5.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('counted_encode'), d.get('huffman_roofline'), d.get('check'))"

timeout -k 10 300 python3 bench.py --workload c5 --steps 10 --warmup 2 --no-cpu --no-e2e --no-decode --no-gop --no-pack-overlap > gpurun_out/c5b.json 2>gpurun_out/c5b.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/c5b.json')); print('no overlap', d['value'], d['ms_per_step'], d['check']['bit_exact'])"
