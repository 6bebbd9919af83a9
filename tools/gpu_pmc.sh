#!/bin/bash
# PMC passes over tools/pmc_probe.py (16 x 4K frames per launch, 8 launches): instruction mix,
# wave occupancy/wait states, LDS bank conflicts.  Args: extra env as NAME=VALUE (e.g. IE_ABLATE=31).
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pmc${TAG:+_$TAG}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p$i -o run -- python3 $R/tools/pmc_probe.py fast 16 > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/p$i.log; exit $rc; fi
done
python3 $R/tools/pmc_summary.py $(find $O -name "*counter_collection.csv") | grep encode_kernel
