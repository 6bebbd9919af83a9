#!/bin/bash
# Round-end GPU session, part 1: every -m gpu test, smoke, the default bench line and the other
# workloads' bench lines.  Each GPU step has its own limit; a fault / abort / timeout ends it.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/final
mkdir -p $O
cd $R
( while sleep 50; do echo "[hb $(date +%T)]"; done ) &
HB=$!
trap 'kill $HB' EXIT
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-1} $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
if [ "${TESTS}" != "none" ]; then
TAILN=3 step pytest timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread
step smoke timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_default timeout -k 10 400 python bench.py
for wl in ${WLS-c3 c4 c5}; do step bench_$wl timeout -k 10 400 python bench.py --workload $wl --steps 10 --warmup 2 --cpu-iters 2; done
exit 0
