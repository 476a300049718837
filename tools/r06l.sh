#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r06l
X=$R/smallz4_amd/lib
bash tools/gpu_steps.sh $O \
 "gen|300|python3 tools/prof_shape.py silesia --reps 1 && python3 tools/prof_shape.py text4m --reps 1" \
 "sil|120|python3 tools/prof_shape.py silesia --reps 3" \
 "pf_sil|120|SMALLZ4_AMD_LIB=$X/libsmallz4_amd_pf.so python3 tools/prof_shape.py silesia --reps 3" \
 "sil2|120|python3 tools/prof_shape.py silesia --reps 3" \
 "pf_sil2|120|SMALLZ4_AMD_LIB=$X/libsmallz4_amd_pf.so python3 tools/prof_shape.py silesia --reps 3" \
 "txt|120|python3 tools/prof_shape.py text4m --reps 3" \
 "pf_txt|120|SMALLZ4_AMD_LIB=$X/libsmallz4_amd_pf.so python3 tools/prof_shape.py text4m --reps 3" \
 "dict|200|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/dict -o run -- python3 $R/tools/time_dict.py 8"
