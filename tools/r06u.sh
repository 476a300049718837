#!/bin/bash
O=gpurun_out/r06u
bash tools/gpu_steps.sh $O \
 "carry|200|python3 tools/time_carry.py" \
 "levels|200|python3 tools/time_levels.py 1 3 6 8 9" \
 "tests|500|python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh gpurun_out/r06u \
 "zu_def|300|python3 tools/prof_shape.py zu" \
 "zu_384|300|SZ4_BATCH_CHUNK=402653184 python3 tools/prof_shape.py zu" \
 "zu_512|300|SZ4_BATCH_CHUNK=536870912 python3 tools/prof_shape.py zu"
