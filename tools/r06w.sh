#!/bin/bash
O=gpurun_out/r06w
bash tools/gpu_steps.sh $O \
 "zu|300|python3 tools/prof_shape.py zu" \
 "shards|600|python -u -m pytest tests/test_shards.py tests/test_memory.py -m gpu -x -v -s --timeout 500 --timeout-method thread"
bash tools/gpu_steps.sh gpurun_out/r06w "diag7|300|python3 tools/diag_fix.py 256"
