# Decode timing of variant libraries (VARS: names under imageencoder_amd/lib/var_*), n in NS, kinds KINDS
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
for rep in 1 2; do for n in ${NS:-4 8}; do for v in $VARS; do
  IE_LIB=imageencoder_amd/lib/var_$v/libie_hip.so timeout -k 10 120 python tools/prof_decode.py $n ${KINDS:-U,flat,ex3} | sed "s/^/$v /" || exit 1
done; done; done
