# encode4w/4p per-wave phase stamps (IE_PROFILE builds) of one NF-frame 4K launch, NF in $NFS, for
# every variant library named in $VARS (imageencoder_amd/lib/var_NAME; default: prof)
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
for v in ${VARS:-prof}; do
for nf in ${NFS:-1 16}; do
  IE_LIB=$R/imageencoder_amd/lib/var_$v/libie_hip.so IE_STAMPS=$R/gpurun_out/st_${v}_$nf.bin NF=$nf SHAPE=${SHAPE:-c2} timeout -k 10 120 python3 $R/tools/stamp_run.py || exit 1
  echo "== $v NF $nf"; python3 $R/tools/${STAMPS_PY:-stamps_w.py} $R/gpurun_out/st_${v}_$nf.bin || exit 1
done
done
