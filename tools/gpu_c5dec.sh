# C5 (counted encode + pack context) tests and bench lines, then the record-decode tests and timings
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
bash tools/gpu_c5.sh || exit 1
bash tools/gpu_dectest.sh || exit 1
