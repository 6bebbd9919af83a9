# decode timing: product build vs a variant (same box), kernel stats of each
for v in prod plain prod; do
  L=imageencoder_amd/lib/libie_hip.so; [ $v = prod ] || L=imageencoder_amd/lib/var_$v/libie_hip.so
  echo "== $v"; IE_LIB=$L timeout -k 10 120 python -u tools/prof_decode.py 4 U,flat 2>&1 | grep R=
done
