#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r06as
bash tools/gpu_steps.sh $O \
 "l6|200|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/l6 -o run -- python3 $R/tools/time_levels.py 6"
