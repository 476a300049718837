#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r06f
bash tools/gpu_steps.sh $O \
 "gen|200|python3 tools/prof_shape.py silesia --reps 1 && python3 tools/prof_shape.py text4m --reps 1" \
 "unlz4_sil|150|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/unlz4_sil -o run -- python3 $R/tools/prof_unlz4.py silesia" \
 "unlz4_txt|150|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/unlz4_txt -o run -- python3 $R/tools/prof_unlz4.py text4m" \
 "e8|120|python3 tools/prof_shape.py enwik8 --reps 5" \
 "tests|400|python -u -m pytest tests/test_unlz4.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread"
