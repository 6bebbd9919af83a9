#!/bin/bash
# Round-end GPU session: every -m gpu test, smoke, the default bench line, the four workloads'
# bench lines, the C2 kernel trace and HBM passes, the decode and P-frame traces.
# Each GPU step has its own limit; a fault / abort / timeout ends the script.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/final
mkdir -p $O
cd $R
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-1} $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
TAILN=3 step pytest timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default timeout -k 10 400 python bench.py
for wl in c3 c4 c5; do step bench_$wl timeout -k 10 400 python bench.py --workload $wl --steps 10 --warmup 2 --cpu-iters 2; done
export TMPDIR=/tmp
BOPT="--steps 10 --warmup 2 --no-cpu --no-single-frame --no-e2e --no-decode --no-gop"
step c2_trace timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 $R/bench.py $BOPT
step pmc_fetch timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py $BOPT
step pmc_write timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py $BOPT
python3 $R/tools/traffic.py encode_kernel $(find $O/pmc_fetch -name "*counter_collection.csv" | head -1) $(find $O/pmc_write -name "*counter_collection.csv" | head -1) $O/traffic_c2.json
step c3_trace timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o run -- python3 $R/bench.py --workload c3 $BOPT
step c5_trace timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o run -- python3 $R/bench.py --workload c5 $BOPT
step dec4_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec4 -o run -- python3 $R/tools/prof_decode.py 4 U,flat
step dec8_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dec8 -o run -- python3 $R/tools/prof_decode.py 8 U,flat
step decode4 timeout -k 10 120 python3 tools/prof_decode.py 4
step decode8 timeout -k 10 120 python3 tools/prof_decode.py 8
step gop timeout -k 10 200 python3 tools/prof_gop.py
step gop_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gop -o run -- python3 $R/tools/prof_gop.py
exit 0
