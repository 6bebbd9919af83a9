#!/bin/bash
# Decode profiling: kernel trace of the 4K 4x4 decode (U, flat) and the table pass's wave stamps.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/decprof; mkdir -p $O; cd $R
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 $R/tools/prof_decode.py ${DEC_N:-4} ${DEC_KINDS:-U,flat} > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
grep "R=" $O/trace.log
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/decprof/tr/run_kernel_stats.csv")):
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.2f} us")
PY
IE_LIB=imageencoder_amd/lib/var_prof/libie_hip.so IE_DEC_STAMPS=$O/st.bin timeout -k 10 120 python3 tools/dec_stamps.py ${DEC_N:-4} U $O/st.bin 2>&1 | grep -v amdgpu.ids
