# Decode parameter sweep (environment overrides of the product build): table-pass chunks per wave
# (IE_REC_TM) and claim-table bits (IE_REC_HB) for 4x4; records per chunk for 8x8
R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
for tm in 1 2 3; do for hb in 6 7 8 9; do
  echo "tm=$tm hb=$hb"; IE_REC_TM=$tm IE_REC_HB=$hb timeout -k 10 120 python tools/prof_decode.py 4 U,M,ex4 || exit 1
done; done
for r in 28 32 36 40; do echo "n8 R=$r"; IE_DEC_R=$r timeout -k 10 120 python tools/prof_decode.py 8 U,M,ex4 || exit 1; done
