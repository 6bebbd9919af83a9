# Huffman pack variants (imageencoder_amd/lib/var_NAME, in LIBS; "product": the in-tree build).
# The Huffman pass runs in libie_host.so, which loads the in-tree libie_hip.so through its rpath
# (IE_LIB would not reach it), so each variant is copied over the in-tree library for its run and
# the original restored: the Huffman GPU tests on each, then the C5 bench's pack / step times,
# alternating twice.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
L=imageencoder_amd/lib/libie_hip.so; cp $L /tmp/libie_hip.orig.so
use() { if [ "$1" = product ]; then cp /tmp/libie_hip.orig.so $L; else cp imageencoder_amd/lib/var_$1/libie_hip.so $L; fi; }
for v in $LIBS; do
  use $v
  timeout -k 10 300 python -u -m pytest tests/test_gpu_files.py tests/test_gpu_stream.py -m gpu -x -q -k "uff or ount" \
    -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pack_$v.log 2>&1 || { echo "tests failed on $v"; tail -5 $O/pack_$v.log; use product; exit 1; }
  echo "$v: $(tail -1 $O/pack_$v.log)"
done
for rep in 1 2; do for v in $LIBS; do
  use $v
  timeout -k 10 200 python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu --no-single-frame --no-e2e --no-decode --no-gop > $O/pack_b_$v.json 2> $O/pack_b_$v.err || { echo "bench failed on $v"; tail -3 $O/pack_b_$v.err; use product; exit 1; }
  python3 -c "import json,sys; d=json.loads([x for x in open(sys.argv[1]) if x.startswith('{')][-1]); h=d['huffman_roofline']; print(sys.argv[2], 'step', d['ms_per_step'], 'pack_us', h['pack_us'], 'hist_us', h['hist_us'], 'enc', d['roofline']['launch_us'])" $O/pack_b_$v.json $v
done; done
use product
