#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r06s
bash tools/gpu_steps.sh $O \
 "l3|200|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/l3 -o run -- python3 $R/tools/time_levels.py 3" \
 "l6|200|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/l6 -o run -- python3 $R/tools/time_levels.py 6" \
 "l8|200|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/l8 -o run -- python3 $R/tools/time_levels.py 8" \
 "tests|500|python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread"
