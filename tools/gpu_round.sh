# C5 + decode checks, then an in-process A/B of the encoder variants named in AB
( while sleep 50; do echo "[hb $(date +%T)]"; done ) &
HB=$!
trap 'kill $HB' EXIT
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
bash tools/gpu_c5dec.sh || exit 1
[ -n "$AB" ] && { TESTS=none AB="$AB" bash tools/gpu_ab.sh || exit 1; }
[ -n "$AB1" ] && { echo "== single 4K frame per launch"; TESTS=none AB="$AB1" ABARGS="--frames 1 --iters 40" bash tools/gpu_ab.sh || exit 1; }
for k in ${C4K}; do
  timeout -k 10 300 python3 bench.py --workload c4 --steps 10 --warmup 2 --no-cpu --chunks $k > gpurun_out/c4k$k.json 2>gpurun_out/c4k$k.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c4 K=$k', d['value'], d['ms_per_step'], d['roofline'])" gpurun_out/c4k$k.json
done
exit 0
