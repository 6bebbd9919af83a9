( while sleep 50; do echo "[hb $(date +%T)]"; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_files.py -m gpu -x -q --timeout 120 --timeout-method thread -k "small_launch or golden or chain_prefix or random_frames or stream" 2>&1 | tail -3 || exit 1
NFS=1 bash tools/gpu_stamps.sh || exit 1
timeout -k 10 300 python3 bench.py --workload c2 --steps 10 --warmup 2 --no-cpu --no-e2e --no-decode --no-gop > gpurun_out/b.json 2>gpurun_out/b.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/b.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('single_frame'), d.get('check'))"
