#!/bin/bash
# round 6 diagnostics: XCD-ordered segments A/B, decoder on 4 MiB blocks, k_find_big / k_find_sorted counters
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r06d
X=$R/smallz4_amd/lib
bash tools/gpu_steps.sh $O \
 "gen|200|python3 tools/prof_shape.py silesia --reps 1 && python3 tools/prof_shape.py text4m --reps 1" \
 "base_sil|120|python3 tools/prof_shape.py silesia --reps 3" \
 "xcd_sil|120|SMALLZ4_AMD_LIB=$X/libsmallz4_amd_xcd.so python3 tools/prof_shape.py silesia --reps 3" \
 "base_txt|120|python3 tools/prof_shape.py text4m --reps 3" \
 "xcd_txt|120|SMALLZ4_AMD_LIB=$X/libsmallz4_amd_xcd.so python3 tools/prof_shape.py text4m --reps 3" \
 "unlz4_sil|150|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/unlz4_sil -o run -- python3 $R/tools/prof_unlz4.py silesia" \
 "unlz4_txt|150|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/unlz4_txt -o run -- python3 $R/tools/prof_unlz4.py text4m" \
 "big_sil|150|python3 tools/diag_big.py 211.93858 silesia" \
 "big_zu|200|python3 tools/diag_big.py 268 zu" \
 "find_zu|200|python3 tools/diag_find.py 268 65535 zu" \
 "find_e8|150|python3 tools/diag_find.py 100 65535 enwik8"
