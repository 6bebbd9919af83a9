# The C4 test's 512-frame single launch: default order, ticket order, the v1 kernel; then the
# gop tests and the C4 test itself (heartbeat: the spawned ranks print nothing for minutes)
( while sleep 50; do echo "[hb $(date +%T)]"; done ) &
HB=$!
trap 'kill $HB' EXIT
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
timeout -k 10 150 python3 -u $R/tools/big_launch.py || exit 1
IE_FORCE_TICKET=1 timeout -k 10 150 python3 -u $R/tools/big_launch.py || exit 1
IE_LIB=$R/imageencoder_amd/lib/var_v1/libie_hip.so IE_FORCE_TICKET=1 timeout -k 10 150 python3 -u $R/tools/big_launch.py || exit 1
timeout -k 10 300 python -u -m pytest $R/tests/test_gop.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
timeout -k 10 620 python -u -m pytest $R/tests/test_gpu_dist.py -m gpu -x -q -k c4_shape --timeout 600 --timeout-method thread || exit 1
