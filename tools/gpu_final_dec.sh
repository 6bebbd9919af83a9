R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/final; mkdir -p $O; cd $R
( while sleep 50; do echo "[hb $(date +%T)]"; done ) &
HB=$!; trap 'kill $HB' EXIT
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-1} $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
export TMPDIR=/tmp
TAILN=20 step decode timeout -k 10 300 bash tools/gpu_decode.sh
TAILN=6 step gop timeout -k 10 200 python3 tools/prof_gop.py
step gop_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gop -o run -- python3 $R/tools/prof_gop.py
step bench_default timeout -k 10 400 python bench.py
step bench_c3 timeout -k 10 400 python bench.py --workload c3 --steps 10 --warmup 2 --cpu-iters 2
exit 0
