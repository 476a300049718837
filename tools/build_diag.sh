#!/bin/bash
# builds the SZ4_DIAG=N variant of the HIP library (3: per-wavefront counters of k_find_sorted, 5: k_find_long9,
# 6: k_find_big's phase clocks, 7: k_dp_fix's repair) as smallz4_amd/lib/libsmallz4_amd_diagN.so
set -e
cd "$(dirname "$0")/../smallz4_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DSZ4_DIAG=${1:-3} -o ../lib/libsmallz4_amd_diag${1:-3}.so sz4_kernels.hip sz4_dict.hip sz4_unlz4.hip sz4_host.cpp
