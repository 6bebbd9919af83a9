#!/bin/bash
# Bench lines of the given workloads (WLS, default c2) -> gpurun_out/bench/<wl>.json, and, with
# TRACE=1, a rocprofv3 kernel trace of a short run of each.  One time limit per GPU step.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/bench; mkdir -p $O; cd $R
export TMPDIR=/tmp
for wl in ${WLS:-c2}; do
  timeout -k 10 ${BT:-400} python3 -u bench.py --workload $wl ${BARGS:---steps 20 --warmup 3} > $O/$wl.json 2> $O/$wl.err
  rc=$?; echo "$wl rc=$rc"; tail -c 1500 $O/$wl.json; echo; [ $rc -eq 0 ] || { tail -5 $O/$wl.err; exit $rc; }
  if [ "${TRACE:-0}" = 1 ]; then
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${wl}_trace -o run -- python3 $R/bench.py --workload $wl --steps 10 --warmup 2 --no-cpu --no-single-frame --no-e2e --no-decode --no-gop > $O/${wl}_trace.log 2>&1) || { echo "trace failed"; tail -3 $O/${wl}_trace.log; exit 1; }
    head -6 $(find $O/${wl}_trace -name "*kernel_stats.csv" | head -1) | cut -c1-200
  fi
done
