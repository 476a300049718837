#!/bin/bash
O=gpurun_out/r06ap
L=smallz4_amd/lib
bash tools/gpu_steps.sh $O \
 "base|200|python3 tools/prof_shape.py enwik8 --reps 10" \
 "dp2048|200|SMALLZ4_AMD_LIB=$L/libsmallz4_amd_dp2048.so python3 tools/prof_shape.py enwik8 --reps 10" \
 "dp8192|200|SMALLZ4_AMD_LIB=$L/libsmallz4_amd_dp8192.so python3 tools/prof_shape.py enwik8 --reps 10" \
 "base2|200|python3 tools/prof_shape.py enwik8 --reps 10"
