R=${GRAFT_REPO_ROOT:-/root/repo}; cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c5t -o run -- python3 $R/bench.py --workload c5 --steps 5 --warmup 1 --no-cpu --no-e2e --no-decode --no-gop --no-single-frame --no-check > $R/gpurun_out/c5t.log 2>&1 || { tail -5 $R/gpurun_out/c5t.log; exit 1; }
python3 $R/tools/trace_grid.py $(find $R/gpurun_out/c5t -name "*kernel_trace.csv") | cut -c1-200
