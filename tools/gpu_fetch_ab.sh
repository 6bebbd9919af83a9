#!/bin/bash
# FETCH_SIZE per launch of the dominant encode kernel for each library in LIBS ("product" = the
# in-tree build, NAME = imageencoder_amd/lib/var_NAME), bench workload WL: one --pmc pass each,
# each under its own time limit -> gpurun_out/fetchab/
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/fetchab; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
WL=${WL:-c4}; K="encode4p_kernel<false>"; G=""; [ $WL = c4 ] && G=2080768
BOPT="--steps 6 --warmup 1 --no-cpu --no-single-frame --no-e2e --no-decode --no-gop --no-check"
for v in ${LIBS:-product}; do
  L=$R/imageencoder_amd/lib/libie_hip.so; [ $v = product ] || L=$R/imageencoder_amd/lib/var_$v/libie_hip.so
  IE_LIB=$L timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/${WL}_$v -o run -- python3 $R/bench.py --workload $WL $BOPT > $O/${WL}_$v.log 2>&1 || { echo "$v fetch failed"; tail -3 $O/${WL}_$v.log; exit 1; }
  f=$(find $O/${WL}_$v -name "*counter_collection.csv" | head -1)
  python3 -c "import sys; sys.path.insert(0, sys.argv[1]); from traffic import mean_counter; v, n = mean_counter(sys.argv[2], sys.argv[3], 'FETCH_SIZE', int(sys.argv[5]) if len(sys.argv) > 5 else None); print(sys.argv[4], 'FETCH_SIZE KiB (raw) per launch', round(v, 1), 'over', n)" $R/tools $f "$K" $v $G
done
