# Table-pass statistics and phase stamps of the record decode (profiling build) per content kind
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
L=$R/imageencoder_amd/lib/var_prof/libie_hip.so
for nk in ${NKS:-4:G 8:G 8:U}; do
  n=${nk%%:*}; k=${nk##*:}
  echo "== n=$n kind=$k"
  IE_LIB=$L IE_DEC_STATS=1 IE_DEC_STAMPS=$O/dec_stamps.bin timeout -k 10 120 python3 tools/dec_stamps.py $n $k $O/dec_stamps.bin 2>&1 | grep -v amdgpu.ids || exit 1
done
