#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r06e
X=$R/smallz4_amd/lib
bash tools/gpu_steps.sh $O \
 "gen|200|python3 tools/prof_shape.py silesia --reps 1 && python3 tools/prof_shape.py text4m --reps 1" \
 "unlz4_sil|150|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/unlz4_sil -o run -- python3 $R/tools/prof_unlz4.py silesia" \
 "unlz4_txt|150|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/unlz4_txt -o run -- python3 $R/tools/prof_unlz4.py text4m" \
 "unlz4_e8|150|python3 tools/prof_unlz4.py enwik8" \
 "new_sil|120|python3 tools/prof_shape.py silesia --reps 3" \
 "ext4_sil|120|SMALLZ4_AMD_LIB=$X/libsmallz4_amd_ext4.so python3 tools/prof_shape.py silesia --reps 3" \
 "old_sil|120|SMALLZ4_AMD_LIB=$X/libsmallz4_amd_old.so python3 tools/prof_shape.py silesia --reps 3" \
 "new_txt|120|python3 tools/prof_shape.py text4m --reps 3" \
 "ext4_txt|120|SMALLZ4_AMD_LIB=$X/libsmallz4_amd_ext4.so python3 tools/prof_shape.py text4m --reps 3" \
 "new_e8|120|python3 tools/prof_shape.py enwik8 --reps 5" \
 "ext4_e8|120|SMALLZ4_AMD_LIB=$X/libsmallz4_amd_ext4.so python3 tools/prof_shape.py enwik8 --reps 5" \
 "old_e8|120|SMALLZ4_AMD_LIB=$X/libsmallz4_amd_old.so python3 tools/prof_shape.py enwik8 --reps 5" \
 "tests|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
