#!/bin/bash
O=gpurun_out/r06r
bash tools/gpu_steps.sh $O \
 "base|200|python3 tools/time_levels.py 3 6 8" \
 "cap64|200|SMALLZ4_AMD_LIB=smallz4_amd/lib/libsmallz4_amd_cap64.so python3 tools/time_levels.py 3 6 8" \
 "cap256|200|SMALLZ4_AMD_LIB=smallz4_amd/lib/libsmallz4_amd_cap256.so python3 tools/time_levels.py 3 6 8"
