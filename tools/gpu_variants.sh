#!/bin/bash
# Correctness on the default library, then the c2 bench for every variant in imageencoder_amd/lib/var_*.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out; mkdir -p $O; cd $R
stop_if_fatal() { local rc=$1; if [ $rc -ge 124 ] || [ $rc -lt 0 ]; then echo "fatal rc=$rc"; exit $rc; fi; }
[ -n "$NOTEST" ] || timeout -k 10 900 python -m pytest tests/test_gpu_encode.py tests/test_gpu_files.py -m gpu -x -q -p no:cacheprovider --timeout 300 > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest_gpu.log; stop_if_fatal $rc; [ $rc -eq 0 ] || exit $rc
for v in imageencoder_amd/lib/var_*; do
  n=$(basename $v)
  IE_LIB=$R/$v/libie_hip.so timeout -k 10 300 python bench.py --workload ${WL:-c2} --steps 20 --warmup 3 --no-cpu > $O/bench_$n.log 2>&1
  rc=$?; echo "$n rc=$rc"; tail -1 $O/bench_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['launch_us'], d['roofline']['frac'], d.get('single_frame'), d['fallback_coefs_per_launch'])" ; stop_if_fatal $rc
done
for ab in ${ABLATES:-}; do
  IE_ABLATE=$ab timeout -k 10 300 python bench.py --workload ${WL:-c2} --steps 20 --warmup 3 --no-cpu > $O/bench_ab$ab.log 2>&1
  rc=$?; echo "ablate $ab rc=$rc"; tail -1 $O/bench_ab$ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['launch_us'])"; stop_if_fatal $rc
done
