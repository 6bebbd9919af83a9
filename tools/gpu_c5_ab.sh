#!/bin/bash
# C5 bench lines (whole step, first-occurrence stage and pack times) of the in-tree build and the
# variants in VARS (imageencoder_amd/lib/var_NAME with its own libie_host.so, through IE_LIB),
# alternating, each run under its own time limit.
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
for i in 1 2; do for v in product ${VARS:-}; do
  L=$R/imageencoder_amd/lib/libie_hip.so; [ $v = product ] || L=$R/imageencoder_amd/lib/var_$v/libie_hip.so
  IE_LIB=$L timeout -k 10 200 python bench.py --workload ${WL:-c5} --steps 10 --warmup 2 --no-cpu --no-single-frame --no-e2e --no-decode --no-gop > /tmp/b.json 2>/tmp/b.err || { tail -5 /tmp/b.err; exit 1; }
  python3 -c "
import json;l=[x for x in open('/tmp/b.json') if x.startswith('{')][-1];d=json.loads(l)
h=d.get('huffman_roofline',{})
print('$v', d['ms_per_step'], d['roofline']['launch_us'], h.get('hist_us'), h.get('pack_us'), d.get('check',{}).get('bit_exact'))"
done; done
