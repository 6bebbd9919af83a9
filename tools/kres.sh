#!/bin/bash
# Resource usage of the encode kernels (VGPRs, scratch, LDS) and scratch-instruction counts.
/opt/rocm/bin/hipcc --offload-arch=gfx950 -mcode-object-version=5 -O3 -std=c++17 -Iinclude -Iimageencoder_amd/csrc -ffp-contract=off --cuda-device-only -S imageencoder_amd/csrc/ie_encode.hip -o build/asm/ie_encode.s "$@" 2>/dev/null
python3 - <<'PY'
import re
s=open('build/asm/ie_encode.s').read()
for m in re.finditer(r'\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel', s, re.S):
    name=m.group(1); body=m.group(2)
    g=lambda k: re.search(k+r'\s+(\d+)', body).group(1)
    k=s[s.index(name+':'):]
    k=k[:k.index('s_endpgm')] if 's_endpgm' in k else k
    nsc=len(re.findall(r'\bscratch_', k))
    print(name[:40], 'vgpr', g('.amdhsa_next_free_vgpr'), 'scratch', g('.amdhsa_private_segment_fixed_size'), 'lds', g('.amdhsa_group_segment_fixed_size'), 'scratch_insts', nsc, 'lines', k.count('\n'))
PY
