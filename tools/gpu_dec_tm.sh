R=${GRAFT_REPO_ROOT:-/root/repo}; cd $R
for tm in 1 2 4 8; do for hb in 0; do
  if [ $hb = 0 ]; then IE_REC_TM=$tm timeout -k 10 120 python tools/prof_decode.py 4 U,M,ex4 || exit 1
  fi; echo "(tm $tm)"; done; done
for tm in 4 8; do for hb in 10 12; do IE_REC_TM=$tm IE_REC_HB=$hb timeout -k 10 120 python tools/prof_decode.py 4 U || exit 1; echo "(tm $tm hb $hb)"; done; done
