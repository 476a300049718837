#!/bin/bash
O=gpurun_out/r06aa
L=smallz4_amd/lib
steps=()
for v in vA vB vC new vE vF vG; do
  if [ $v = new ]; then lib=$L/libsmallz4_amd.so; else lib=$L/libsmallz4_amd_$v.so; fi
  steps+=("${v}_sil|200|SMALLZ4_AMD_LIB=$lib python3 tools/prof_unlz4.py silesia --reps 10")
  steps+=("${v}_txt|200|SMALLZ4_AMD_LIB=$lib python3 tools/prof_unlz4.py text4m --reps 10")
done
bash tools/gpu_steps.sh $O "${steps[@]}"
