# Record-decode chunking A/B (IE_REC_TM chunks per table wave x IE_DEC_R records per chunk), interleaved runs
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
for rep in 1 2 3; do for cfg in ${CFGS:-"2 24" "3 24"}; do
  set -- $cfg
  echo "tm=$1 R=$2: $(IE_REC_TM=$1 IE_DEC_R=$2 IE_HDR_BITS=165 timeout -k 10 60 python3 tools/prof_decode.py 4 G,M,ex4 2>/dev/null | awk '{print $4, $7}' | tr '\n' ' ')" || exit 1
done; done
