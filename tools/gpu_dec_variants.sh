# decode timing per records-per-chunk setting (IE_DEC_R), same box
for r in 32 64 24; do echo "== n8 R=$r"; IE_DEC_R=$r timeout -k 10 120 python -u tools/prof_decode.py 8 2>&1 | grep R=; done
for r in 32 48; do echo "== n4 R=$r"; IE_DEC_R=$r timeout -k 10 120 python -u tools/prof_decode.py 4 2>&1 | grep R=; done
