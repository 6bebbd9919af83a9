# Huffman decode (device-resident) against the walk chunk (IE_HUF_CHUNK bits)
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
for rep in 1 2; do for c in ${CS:-1024 2048 4096 8192}; do
  IE_HUF_CHUNK=$c timeout -k 10 120 python tools/prof_hufdec.py | sed "s/^/chunk=$c /" || exit 1
done; done
