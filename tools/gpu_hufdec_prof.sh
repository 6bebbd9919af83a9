# Kernel trace of the device-resident Huffman decode (tools/prof_hufdec.py) on the in-tree build.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/hufprof; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/tools/prof_hufdec.py > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
tail -1 $O/run.log
f=$(find $O -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | head -14
