set -o pipefail
mkdir -p gpurun_out
( while sleep 50; do echo "[hb $(date +%T)]"; done ) &
HB=$!
trap 'kill $HB' EXIT
REPS=2 timeout -k 10 150 python3 -u tools/big_launch.py || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; r=$?; tail -3 gpurun_out/gpu_tests.log; [ $r -eq 0 ] || exit $r
cd /tmp && export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/sf -o run -- python3 $R/bench.py --workload c2 --steps 3 --warmup 1 --no-cpu --no-e2e --no-decode --no-gop --no-check > $R/gpurun_out/sf.log 2>&1 || exit 1
python3 $R/tools/trace_grid.py $(find $R/gpurun_out/sf -name "*kernel_trace.csv") encode
exit 0
