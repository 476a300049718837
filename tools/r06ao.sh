#!/bin/bash
O=gpurun_out/r06ao
bash tools/gpu_steps.sh $O \
 "dict|200|python3 tools/time_dict.py 8" \
 "bench|600|python3 bench.py --no-shapes --no-levels --no-stream --cpu-seconds 1"
