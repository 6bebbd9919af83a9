#!/bin/bash
# Round-6 GPU session driver: TESTS (pytest -m gpu files, "none" to skip), then A/B lines given as
# AB1..AB4 (each: "[ab.py args] lib[@ENV=VAL] ..." with "product" for the in-tree build and
# "var:NAME" for imageencoder_amd/lib/var_NAME).  Every GPU step has its own time limit and the
# first failure ends the script.
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
export TMPDIR=/tmp
TESTS=${TESTS:-tests/test_gpu_encode.py}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-500} python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2 3 4 5 6; do
  v=AB$i; line=${!v}; [ -z "$line" ] && continue
  args=""; libs=""
  for tok in $line; do
    case $tok in
      --*|[0-9]*) args="$args $tok";;
      product*) libs="$libs imageencoder_amd/lib/libie_hip.so${tok#product}";;
      var:*) t=${tok#var:}; libs="$libs imageencoder_amd/lib/var_${t%%@*}/libie_hip.so$( [[ $t == *@* ]] && echo "@${t#*@}")";;
      *) args="$args $tok";;
    esac
  done
  echo "== AB$i:$args"
  timeout -k 10 300 python -u tools/ab.py --rounds ${ROUNDS:-9} $args $libs > $O/ab$i.log 2>&1
  rc=$?; grep -v "^running\|FP64" $O/ab$i.log | tail -14; [ $rc -eq 0 ] || { echo "ab rc=$rc"; tail -20 $O/ab$i.log; exit $rc; }
done
