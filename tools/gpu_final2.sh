#!/bin/bash
# Round-end GPU session, part 2: HBM traffic + kernel traces of the four workloads, decode / Huffman
# decode / P-frame traces and timings, the encoder's phase stamps and PMC instruction mix.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/final
mkdir -p $O
cd $R
( while sleep 50; do echo "[hb $(date +%T)]"; done ) &
HB=$!
trap 'kill $HB' EXIT
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-1} $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
export TMPDIR=/tmp
step traffic timeout -k 10 700 bash tools/gpu_traffic.sh
TAILN=20 step decode timeout -k 10 300 bash tools/gpu_decode.sh
TAILN=4 step hufdec timeout -k 10 120 python3 tools/prof_hufdec.py
step hufdec_trace timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hufdec -o run -- python3 $R/tools/prof_hufdec.py
TAILN=6 step gop timeout -k 10 200 python3 tools/prof_gop.py
step gop_trace timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gop -o run -- python3 $R/tools/prof_gop.py
TAILN=30 step stamps env NFS="1 16" timeout -k 10 300 bash tools/gpu_stamps.sh
TAILN=40 step pmc env LIBS="imageencoder_amd/lib/libie_hip.so imageencoder_amd/lib/var_v1/libie_hip.so" timeout -k 10 400 bash tools/gpu_pmc_insts.sh
TAILN=6 step ab_single env TESTS=none AB="product r02" ABARGS="--frames 1 --iters 40" timeout -k 10 300 bash tools/gpu_ab.sh
exit 0
