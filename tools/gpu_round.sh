#!/bin/bash
# One GPU session: tests, benches for every workload, rocprof kernel stats and HBM PMC passes.
# Every GPU step has its own time limit; a fault / abort / timeout ends the script.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
mkdir -p $O
cd $R
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
stop_if_fatal() { local rc=$1; if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then echo "fatal rc=$rc"; exit $rc; fi; }

if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 $O/pytest_gpu.log; stop_if_fatal $rc; ok $rc || exit $rc
fi

for wl in c2 c3 c4 c5; do
  timeout -k 10 400 python bench.py --workload $wl --steps 10 --warmup 2 --cpu-iters 2 > $O/bench_$wl.log 2>&1
  rc=$?; echo "bench $wl rc=$rc"; tail -1 $O/bench_$wl.log; stop_if_fatal $rc; [ $rc -eq 0 ] || exit $rc
done

cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stats -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-single-frame --no-e2e --no-decode --no-gop > $O/prof_stats.log 2>&1
rc=$?; echo "rocprof stats rc=$rc"; stop_if_fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-single-frame --no-e2e --no-decode --no-gop > $O/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; stop_if_fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-single-frame --no-e2e --no-decode --no-gop > $O/pmc_write.log 2>&1
rc=$?; echo "pmc write rc=$rc"; stop_if_fatal $rc
find $O/prof_stats $O/pmc_fetch $O/pmc_write -name "*.csv" | head -20
python3 $R/tools/traffic.py encode_kernel $(find $O/pmc_fetch -name "*counter_collection.csv" | head -1) $(find $O/pmc_write -name "*counter_collection.csv" | head -1) $O/traffic_c2.json
timeout -k 10 120 python3 $R/tools/prof_decode.py 4 > $O/decode4.txt 2>&1 && timeout -k 10 120 python3 $R/tools/prof_decode.py 8 > $O/decode8.txt 2>&1
rc=$?; echo "decode timings rc=$rc"; grep R= $O/decode4.txt $O/decode8.txt
exit 0
