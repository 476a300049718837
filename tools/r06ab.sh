#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r06ab
bash tools/gpu_steps.sh $O \
 "tests|400|python -u -m pytest tests/test_unlz4.py -m gpu -x -q --timeout 300 --timeout-method thread" \
 "sil|200|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/sil -o run -- python3 $R/tools/prof_unlz4.py silesia" \
 "txt|200|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/txt -o run -- python3 $R/tools/prof_unlz4.py text4m"
