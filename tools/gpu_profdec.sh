#!/bin/bash
# per-kernel times of the decode (rocprofv3 kernel trace) for block size $1
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/profdec$1 -o run -- python3 $R/tools/prof_decode.py $1 > $R/gpurun_out/profdec$1.log 2>&1
f=$(find $R/gpurun_out/profdec$1 -name '*kernel_stats.csv' | head -1)
cut -d, -f1-8 "$f" | head -20
