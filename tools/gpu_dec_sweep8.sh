# 8x8 decode against the records per chunk (IE_DEC_R)
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
for r in ${RS:-20 24 26 28 30 32}; do echo "n8 R=$r"; IE_DEC_R=$r timeout -k 10 120 python tools/prof_decode.py 8 ${KINDS:-U,M,grad,flat,ex1,ex4} || exit 1; done
