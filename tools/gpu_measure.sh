#!/bin/bash
# Measurement session: kernel traces (STEPS, default: C3, C5 and the 4K decode) into gpurun_out/meas,
# then the bench lines of C3 and C5.  Every GPU step has its own limit; a failure ends the script.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/meas; mkdir -p $O; cd $R
set -o pipefail
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
export TMPDIR=/tmp
BOPT="--steps 10 --warmup 2 --no-cpu --no-single-frame --no-e2e --no-decode --no-gop"
STEPS=${STEPS:-"c3_trace c5_trace dec4_trace c3_bench c5_bench"}
for s in $STEPS; do case $s in
  c3_trace) step c3_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- python3 $R/bench.py --workload c3 $BOPT ;;
  c5_trace) step c5_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o run -- python3 $R/bench.py --workload c5 $BOPT ;;
  dec4_trace) step dec4_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec4 -o run -- python3 $R/tools/prof_decode.py 4 U,flat ;;
  c3_bench) step c3_bench timeout -k 10 400 python3 bench.py --workload c3 --steps 10 --warmup 2 --no-cpu ;;
  c5_bench) step c5_bench timeout -k 10 400 python3 bench.py --workload c5 --steps 10 --warmup 2 --no-cpu ;;
esac; done
exit 0
