#!/bin/bash
# Huffman-decode tests on the product build, then tools/prof_hufdec.py for each library in LIBS
# (imageencoder_amd/lib/var_NAME; "product": the in-tree build), alternating.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_files.py tests/test_integration.py -m gpu -x -q -p no:cacheprovider -k "${TK:-huffman or Huffman or decoder or Decoder}" --timeout 120 --timeout-method thread > $O/pytest_huf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_huf.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in ${LIBS:-product}; do
  L=$R/imageencoder_amd/lib/libie_hip.so; [ $v = product ] || L=$R/imageencoder_amd/lib/var_$v/libie_hip.so
  echo "== $v $(IE_LIB=$L timeout -k 10 120 python3 tools/prof_hufdec.py 2>&1 | grep -v amdgpu.ids | tail -1)" || exit 1
done; done
