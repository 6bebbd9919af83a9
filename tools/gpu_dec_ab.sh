#!/bin/bash
# Record-decode tests on the product build, then tools/prof_decode.py (4x4 and 8x8 4K content) for
# each library in LIBS (imageencoder_amd/lib/var_NAME; "product": the in-tree build), alternating.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
[ "${TK:-x}" = none ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_files.py tests/test_gop.py tests/test_integration.py -m gpu -x -q -p no:cacheprovider -k "${TK:-decode or gop or Decoder or decoder}" --timeout 120 --timeout-method thread > $O/pytest_dec.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_dec.log 2>/dev/null; [ $rc -eq 0 ] || exit $rc
# a variant "NAME@ENV=VAL,ENV2=VAL" runs with those environment variables
for i in 1 2; do for tok in ${LIBS:-product}; do
  v=${tok%%@*}; envs=""; [[ $tok == *@* ]] && envs=${tok#*@}
  L=$R/imageencoder_amd/lib/libie_hip.so; [ $v = product ] || L=$R/imageencoder_amd/lib/var_$v/libie_hip.so
  echo "== $tok"
  env ${envs//,/ } IE_LIB=$L IE_HDR_BITS=165 timeout -k 10 120 python3 tools/prof_decode.py 4 ${K4:-G,M,ex4} 2>&1 | grep -v amdgpu.ids || exit 1
  [ "${K8:-G}" = none ] || env ${envs//,/ } IE_LIB=$L IE_HDR_BITS=549 timeout -k 10 120 python3 tools/prof_decode.py 8 ${K8:-G} 2>&1 | grep -v amdgpu.ids || exit 1
done; done
