#!/bin/bash
# Per-phase instruction mix of the C2 encode: the IE_PROFILE build with sections ablated at run time
# (IE_ABLATE bits: 1 no FP64 fix, 2 no emission, 4 no look-back, 8 no store, 16 no FP32 transform,
# 128 no pixel loads), one rocprofv3 --pmc pass each.  Outputs of ablated runs are wrong by design.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmca; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export IE_LIB=$R/imageencoder_amd/lib/var_prof/libie_hip.so
for ab in ${ABLATES:-0 1 2 4 8 16 128 15}; do
  IE_ABLATE=$ab timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $O/a$ab -o run -- python3 $R/tools/pmc_probe.py fast 16 > $O/a$ab.log 2>&1
  rc=$?; echo "ablate $ab rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $O/a$ab.log; exit $rc; fi
done
for ab in ${ABLATES:-0 1 2 4 8 16 128 15}; do
  echo "== ablate $ab"; python3 $R/tools/pmc_summary.py $(find $O/a$ab -name "*counter_collection.csv") | grep "encode_kernel" | grep -v meta
done > $O/summary.txt
cat $O/summary.txt
exit 0
