# encode4w per-wave phase stamps (IE_PROFILE build) of one NF-frame 4K launch, NF in $NFS
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
for nf in ${NFS:-1 16}; do
  IE_LIB=$R/imageencoder_amd/lib/var_prof/libie_hip.so IE_STAMPS=$R/gpurun_out/st$nf.bin NF=$nf timeout -k 10 120 python3 $R/tools/stamp_run.py || exit 1
  echo "== NF $nf"; python3 $R/tools/stamps_w.py $R/gpurun_out/st$nf.bin || exit 1
done
