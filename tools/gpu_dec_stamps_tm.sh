cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for cfg in "2 8" "4 9" "8 10" "8 9"; do set -- $cfg
  echo "== tm=$1 hb=$2"
  IE_REC_TM=$1 IE_REC_HB=$2 timeout -k 10 100 python3 tools/prof_decode.py 4 U 2>&1 | grep -v amdgpu.ids
  IE_REC_TM=$1 IE_REC_HB=$2 IE_LIB=imageencoder_amd/lib/var_prof/libie_hip.so IE_DEC_STAMPS=gpurun_out/st.bin timeout -k 10 100 python3 tools/dec_stamps.py 4 U gpurun_out/st.bin 2>&1 | grep -v "amdgpu.ids\|alive\|start times" || exit 1
done
