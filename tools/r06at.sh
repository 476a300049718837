#!/bin/bash
O=gpurun_out/r06at
L=smallz4_amd/lib
bash tools/gpu_steps.sh $O \
 "base|200|python3 tools/prof_unlz4.py enwik8 --reps 20" \
 "ring8k|200|SMALLZ4_AMD_LIB=$L/libsmallz4_amd_ring8k.so python3 tools/prof_unlz4.py enwik8 --reps 20" \
 "base2|200|python3 tools/prof_unlz4.py enwik8 --reps 20" \
 "ring8k2|200|SMALLZ4_AMD_LIB=$L/libsmallz4_amd_ring8k.so python3 tools/prof_unlz4.py enwik8 --reps 20"
