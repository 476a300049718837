#!/bin/bash
# builds the SZ4_DIAG=3 variant of the HIP library (per-wavefront counters of k_find_sorted)
set -e
cd "$(dirname "$0")/../smallz4_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DSZ4_DIAG=${1:-3} -o ../lib/libsmallz4_amd_diag.so sz4_kernels.hip sz4_dict.hip sz4_unlz4.hip sz4_host.cpp
