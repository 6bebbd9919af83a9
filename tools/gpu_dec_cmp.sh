#!/bin/bash
# Decode: the exact-parse tests, then a kernel trace of the 4K decode (product build), then the
# A/B of variant libraries named in AB (imageencoder_amd/lib/var_NAME) by wall time per call.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/deccmp; mkdir -p $O; cd $R
export TMPDIR=/tmp
if [ "${TESTS:-x}" != "none" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_files.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 $R/tools/prof_decode.py ${DEC_N:-4} ${KINDS:-U,flat} > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
grep "R=" $O/trace.log
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/deccmp/tr/run_kernel_stats.csv")):
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.2f} us")
PY
for v in base $AB; do
  lib=imageencoder_amd/lib/libie_hip.so; [ $v = base ] || lib=imageencoder_amd/lib/var_$v/libie_hip.so
  for n in 4 8; do IE_LIB=$lib timeout -k 10 120 python3 tools/prof_decode.py $n ${KINDS:-U,M,flat} 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || exit 1; done
done
if [ -n "$STAMPS" ]; then
  IE_LIB=imageencoder_amd/lib/var_prof/libie_hip.so IE_DEC_STAMPS=$O/st.bin timeout -k 10 120 python3 tools/dec_stamps.py 4 U $O/st.bin 2>&1 | grep -v amdgpu.ids
fi
