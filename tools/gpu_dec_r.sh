# Decode timing against the records per chunk (IE_DEC_R in RS), n in NS, kinds KINDS
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
for rep in 1 2; do for n in ${NS:-4 8}; do for r in ${RS:-16 24 32 48}; do
  IE_DEC_R=$r timeout -k 10 120 python tools/prof_decode.py $n ${KINDS:-U,M,flat,ex4} || exit 1
done; done; done
