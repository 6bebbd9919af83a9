#!/bin/bash
# Build libie_hip.so variants with extra compile flags: tools/variants.sh NAME "FLAGS" [NAME "FLAGS" ...]
# -> imageencoder_amd/lib/var_NAME/libie_hip.so  (load with IE_LIB=that path); objects in build/
set -e
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  d=build/var_$name; mkdir -p $d
  for k in ie_encode ie_huffman ie_decode ie_pframe ie_capi; do
    src=imageencoder_amd/csrc/$k.hip; [ -f $src ] || src=imageencoder_amd/csrc/$k.cpp
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -mcode-object-version=5 -O3 -std=c++17 -fPIC -Iinclude -Iimageencoder_amd/csrc -ffp-contract=off $flags -c $src -o $d/$k.o &
  done
  wait
  L=imageencoder_amd/lib/var_$name; mkdir -p $L
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $d/*.o -o $L/libie_hip.so
  # the host library beside it, bound to this build (rpath $ORIGIN; imageencoder_amd loads it
  # when IE_LIB points here)
  g++ -shared -fopenmp build/host/*.o -L$L -lie_hip -Wl,-rpath,'$ORIGIN' -o $L/libie_host.so
  echo "built $L/libie_hip.so ($flags)"
done
