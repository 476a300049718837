#!/bin/bash
O=gpurun_out/r06t
bash tools/gpu_steps.sh $O \
 "carry|200|python3 tools/time_carry.py" \
 "levels|200|python3 tools/time_levels.py 1 3 6 8 9" \
 "tests|500|python -u -m pytest tests/test_gpu.py tests/test_stream.py -m gpu -x -q --timeout 300 --timeout-method thread"
