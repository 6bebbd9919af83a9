cd ${GRAFT_REPO_ROOT:-/root/repo}
bash tools/_ab2.sh
ABS="0" bash tools/gpu_stamps.sh 2>&1 | tail -14
