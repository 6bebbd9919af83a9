# Record decode timing (tools/prof_decode.py) of 4x4 / 8x8 4K frames, kernel traces of the golden
# frame's decode -> gpurun_out/dec/, and the C3 bench line's decode leg
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/dec; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
IE_HDR_BITS=165 timeout -k 10 120 python3 $R/tools/prof_decode.py 4 G,U,M,ex4 || exit 1
IE_HDR_BITS=549 timeout -k 10 120 python3 $R/tools/prof_decode.py 8 G,U,M,ex1 || exit 1
for n in 4 8; do
  hb=165; [ $n = 8 ] && hb=549
  IE_HDR_BITS=$hb timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$n -o run -- python3 $R/tools/prof_decode.py $n G > $O/t$n.log 2>&1 || { tail -3 $O/t$n.log; exit 1; }
  cp $(find $O/t$n -name "*kernel_stats.csv" | head -1) $O/${ROUND:-r05}_dec${n}_kernel_stats.csv
  python3 $R/tools/trace_grid.py $(find $O/t$n -name "*kernel_trace.csv" | head -1) rec_ || exit 1
done
timeout -k 10 300 python3 $R/bench.py --workload c3 --steps 3 --warmup 1 --no-cpu --no-e2e --no-gop --no-single-frame > $O/c3.json 2> $O/c3.err || exit 1
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c3 bench decode', d['decode_one_image'])" $O/c3.json
