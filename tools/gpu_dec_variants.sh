# decode timing: product build vs variants (same box)
for v in prod head k24 k6 prod head; do
  L=imageencoder_amd/lib/libie_hip.so; [ $v = prod ] || L=imageencoder_amd/lib/var_$v/libie_hip.so
  echo "== $v"; IE_LIB=$L timeout -k 10 120 python -u tools/prof_decode.py 4 U,M,flat 2>&1 | grep R=
done
