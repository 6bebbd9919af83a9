# P-frame timing (tools/prof_gop.py) of variant libraries (VARS), the reference binary skipped
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
for rep in 1 2; do for v in $VARS; do
  IE_NO_REF=1 IE_LIB=imageencoder_amd/lib/var_$v/libie_hip.so timeout -k 10 120 python tools/prof_gop.py | sed "s/^/$v /" || exit 1
done; done
