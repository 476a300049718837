#!/bin/bash
O=gpurun_out/r06z
L=smallz4_amd/lib
steps=()
for v in head new ring2048 ring1024; do
  if [ $v = new ]; then lib=$L/libsmallz4_amd.so; else lib=$L/libsmallz4_amd_$v.so; fi
  steps+=("${v}_sil|200|SMALLZ4_AMD_LIB=$lib python3 tools/prof_unlz4.py silesia")
  steps+=("${v}_txt|200|SMALLZ4_AMD_LIB=$lib python3 tools/prof_unlz4.py text4m")
done
bash tools/gpu_steps.sh $O "${steps[@]}" \
 "tests|400|python -u -m pytest tests/test_unlz4.py -m gpu -x -q --timeout 300 --timeout-method thread"
