#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r06n
bash tools/gpu_steps.sh $O \
 "tests|500|python -u -m pytest tests/test_gpu.py tests/test_stream.py -m gpu -x -q --timeout 300 --timeout-method thread" \
 "levels|200|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/levels -o run -- python3 $R/tools/time_levels.py 1 3 6 8 9" \
 "dict|200|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/dict -o run -- python3 $R/tools/time_dict.py 8"
