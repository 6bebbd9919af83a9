cd ${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 300 python tools/ab.py ${ABARGS:-} $(ls -d imageencoder_amd/lib/var_*/libie_hip.so) 2>&1 | grep -v amdgpu.ids
