#!/bin/bash
# Measurement session (round 3): kernel traces of C3, C5 and the 4K decode; the C3 streamed-path
# timing inside the bench process against the standalone tool; per-launch time against batch size.
# Every GPU step has its own limit; a failure ends the script.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/meas; mkdir -p $O; cd $R
set -o pipefail
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 $O/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
export TMPDIR=/tmp
BOPT="--steps 10 --warmup 2 --no-cpu --no-single-frame --no-e2e --no-decode --no-gop"
step c3_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- python3 $R/bench.py --workload c3 $BOPT
step c5_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o run -- python3 $R/bench.py --workload c5 $BOPT
step dec4_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec4 -o run -- python3 $R/tools/prof_decode.py 4 U,flat
step c3_bench timeout -k 10 400 python3 bench.py --workload c3 --steps 10 --warmup 2 --no-cpu --no-decode --no-gop
step e2e8 env E2E_N=8 timeout -k 10 300 python3 tools/e2e.py 8
step e2e8_torch env E2E_N=8 E2E_TORCH_STREAM=1 timeout -k 10 300 python3 tools/e2e.py 8
for f in 16 24 32 64; do step batch$f timeout -k 10 200 python3 tools/ab.py --rounds 5 --frames $f imageencoder_amd/lib/libie_hip.so; done
exit 0
