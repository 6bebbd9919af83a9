#!/bin/bash
# Round-end GPU session, part 2: HBM traffic + kernel traces of the four workloads, decode / Huffman
# decode / P-frame traces and timings, the encoder's phase stamps and PMC counters.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/final
mkdir -p $O
cd $R
( while sleep 50; do echo "[hb $(date +%T)]"; done ) &
HB=$!
trap 'kill $HB' EXIT
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-1} $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
export TMPDIR=/tmp
export ROUND=${ROUND:-r06}
if [ "${TRAFFIC:-1}" = 1 ]; then step traffic timeout -k 10 900 bash tools/gpu_traffic.sh; fi
if [ "${FUZZ:-1}" = 1 ]; then
  TAILN=3 step fuzz4 timeout -k 10 700 python3 tools/fuzz_exact.py --n 4 --blocks 1e9 --budget 600 --out $O/${ROUND}_fuzz_4x4.json
  TAILN=3 step fuzz8 timeout -k 10 700 python3 tools/fuzz_exact.py --n 8 --blocks 1e9 --budget 600 --out $O/${ROUND}_fuzz_8x8.json
fi
TAILN=20 step decode timeout -k 10 300 bash tools/gpu_decode.sh
TAILN=4 step hufdec timeout -k 10 120 python3 tools/prof_hufdec.py
step hufdec_trace timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hufdec -o run -- python3 $R/tools/prof_hufdec.py
TAILN=6 step gop timeout -k 10 200 python3 tools/prof_gop.py
step gop_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gop -o run -- python3 $R/tools/prof_gop.py
TAILN=30 step stamps env NFS="1 16" timeout -k 10 300 bash tools/gpu_stamps.sh
TAILN=30 step stamps_c4 env NFS=64 SHAPE=c4 timeout -k 10 300 bash tools/gpu_stamps.sh
TAILN=12 step pmc_insts env LIBS="imageencoder_amd/lib/libie_hip.so" timeout -k 10 200 bash tools/gpu_pmc_valu.sh
TAILN=12 step pmc_util env COUNTERS="SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT" LIBS="imageencoder_amd/lib/libie_hip.so" timeout -k 10 200 bash tools/gpu_pmc_valu.sh
exit 0
