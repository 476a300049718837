#!/bin/bash
O=gpurun_out/r06au
bash tools/gpu_steps.sh $O \
 "levels|200|python3 tools/time_levels.py 1 3 6 --reps 5" \
 "tests|600|python -u -m pytest tests/test_gpu.py tests/test_stream.py -m gpu -x -q --timeout 500 --timeout-method thread"
