#!/bin/bash
O=gpurun_out/r06ah
L=smallz4_amd/lib
bash tools/gpu_steps.sh $O \
 "head_sil|200|SMALLZ4_AMD_LIB=$L/libsmallz4_amd_head.so python3 tools/prof_unlz4.py silesia --reps 10" \
 "new_sil|200|python3 tools/prof_unlz4.py silesia --reps 10" \
 "head_txt|200|SMALLZ4_AMD_LIB=$L/libsmallz4_amd_head.so python3 tools/prof_unlz4.py text4m --reps 10" \
 "new_txt|200|python3 tools/prof_unlz4.py text4m --reps 10" \
 "diag|300|python3 tools/diag_unlz4.py silesia" \
 "tests|400|python -u -m pytest tests/test_unlz4.py -m gpu -x -q --timeout 300 --timeout-method thread"
