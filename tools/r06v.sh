#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r06v
bash tools/gpu_steps.sh $O \
 "zu384|300|cd /tmp && SZ4_BATCH_CHUNK=402653184 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/zu384 -o run -- python3 $R/tools/prof_shape.py zu --reps 1" \
 "zudef|300|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/zudef -o run -- python3 $R/tools/prof_shape.py zu --reps 1"
