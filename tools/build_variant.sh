#!/bin/bash
# builds a tuning variant of the HIP library: tools/build_variant.sh NAME "-DSZ4_X=..." -> lib/libsmallz4_amd_NAME.so
# (select it with SMALLZ4_AMD_LIB=smallz4_amd/lib/libsmallz4_amd_NAME.so)
set -e
cd "$(dirname "$0")/../smallz4_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared $2 -o ../lib/libsmallz4_amd_$1.so sz4_kernels.hip sz4_dict.hip sz4_unlz4.hip sz4_host.cpp
