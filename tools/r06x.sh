#!/bin/bash
O=gpurun_out/r06x
bash tools/gpu_steps.sh $O \
 "diag7|300|python3 tools/diag_fix.py 256" \
 "zu|300|python3 tools/prof_shape.py zu" \
 "zu1g|300|SZ4_BATCH_CHUNK=1610612736 python3 tools/prof_shape.py zu" \
 "tests|600|python -u -m pytest tests/test_gpu.py tests/test_shards.py -m gpu -x -q --timeout 500 --timeout-method thread"
