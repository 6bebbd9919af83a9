#!/bin/bash
# This round's HBM traffic (FETCH_SIZE / WRITE_SIZE, separate --pmc passes) and kernel traces of the
# four workloads' bench runs -> gpurun_out/traffic/<ROUND>_traffic_<wl>.json + *_kernel_stats.csv.
# Each GPU step has its own limit; a failing step ends the script.
R=${GRAFT_REPO_ROOT:-/root/repo}
ROUND=${ROUND:-r06}
O=$R/gpurun_out/traffic; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
BOPT="--steps 6 --warmup 1 --no-cpu --no-single-frame --no-e2e --no-decode --no-gop --no-check"
for wl in ${WLS:-c2 c3 c4 c5}; do
  case $wl in
    c3) K=encode_kernel; G="";;
    c4) K="encode4p_kernel<false>"; G=2080768;;  # the 64-frame launches: 64 x ceil(32400 groups / 256) tiles x 256 threads
    c5) K="encode4p_kernel<true>"; G="";;        # the counting encoder the C5 step runs
    *)  K="encode4p_kernel<false>"; G="";;
  esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${wl}_trace -o run -- python3 $R/bench.py --workload $wl $BOPT > $O/${wl}_trace.log 2>&1 || { echo "$wl trace failed"; tail -3 $O/${wl}_trace.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/${wl}_fetch -o run -- python3 $R/bench.py --workload $wl $BOPT > $O/${wl}_fetch.log 2>&1 || { echo "$wl fetch failed"; tail -3 $O/${wl}_fetch.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/${wl}_write -o run -- python3 $R/bench.py --workload $wl $BOPT > $O/${wl}_write.log 2>&1 || { echo "$wl write failed"; tail -3 $O/${wl}_write.log; exit 1; }
  python3 $R/tools/traffic.py "$K" $(find $O/${wl}_fetch -name "*counter_collection.csv" | head -1) $(find $O/${wl}_write -name "*counter_collection.csv" | head -1) $O/${ROUND}_traffic_${wl}.json $G | cut -c1-300
  cp $(find $O/${wl}_trace -name "*kernel_stats.csv" | head -1) $O/${ROUND}_${wl}_kernel_stats.csv
done
exit 0
