# Huffman decode tests and timing (device-resident) with a kernel trace
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_files.py tests/test_integration.py -m gpu -x -q --timeout 120 --timeout-method thread -k "huffman or decode" 2>&1 | tail -2 || exit 1
timeout -k 10 120 python3 tools/prof_hufdec.py 2>&1 | grep -v amdgpu.ids || exit 1
cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/hufdec -o run -- python3 $R/tools/prof_hufdec.py > $R/gpurun_out/hufdec.log 2>&1 || exit 1
cut -d, -f1-4 $(find $R/gpurun_out/hufdec -name "*kernel_stats.csv" | head -1) | head -12
