# C5 bench lines (Huffman pass timing) of variant libraries (VARS).  The Huffman pass runs in
# libie_host.so, which loads the in-tree libie_hip.so through its rpath (IE_LIB would not reach
# it), so each variant is copied over the in-tree library for its run and the original restored.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
L=imageencoder_amd/lib/libie_hip.so; cp $L /tmp/libie_hip.orig.so
for i in 1 2; do for v in ${VARS:-base}; do
cp imageencoder_amd/lib/var_$v/libie_hip.so $L
timeout -k 10 200 python bench.py --workload c5 --steps 10 --warmup 2 --no-cpu --no-single-frame --no-e2e --no-decode --no-gop > /tmp/b.json 2>/tmp/b.err || { tail -5 /tmp/b.err; cp /tmp/libie_hip.orig.so $L; exit 1; }
python3 -c "
import json;l=[x for x in open('/tmp/b.json') if x.startswith('{')][-1];d=json.loads(l)
h=d.get('huffman_roofline',{})
print('$v', d['ms_per_step'], h.get('hist_us'), h.get('pack_us'), d.get('check',{}).get('bit_exact'))"
done; done
cp /tmp/libie_hip.orig.so $L
