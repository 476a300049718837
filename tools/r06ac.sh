#!/bin/bash
O=gpurun_out/r06ac
bash tools/gpu_steps.sh $O \
 "base|200|python3 tools/time_levels.py 3 8 --reps 5" \
 "cap64|200|SMALLZ4_AMD_LIB=smallz4_amd/lib/libsmallz4_amd_cap64.so python3 tools/time_levels.py 3 8 --reps 5" \
 "cap128|200|SMALLZ4_AMD_LIB=smallz4_amd/lib/libsmallz4_amd_cap128.so python3 tools/time_levels.py 3 8 --reps 5" \
 "base2|200|python3 tools/time_levels.py 3 8 --reps 5"
