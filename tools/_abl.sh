cd ${GRAFT_REPO_ROOT:-/root/repo}
export NOTEST=1 ABLATES="0 1 2 4 8 16 6 14 30 31"
bash tools/gpu_variants.sh && bash tools/gpu_pmc.sh && ABS="0" bash tools/gpu_stamps.sh
