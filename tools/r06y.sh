#!/bin/bash
O=gpurun_out/r06y
bash tools/gpu_steps.sh $O \
 "sil|300|python3 tools/prof_shape.py silesia" \
 "text4m|300|python3 tools/prof_shape.py text4m" \
 "e8|300|python3 tools/prof_shape.py enwik8" \
 "tests|600|python -u -m pytest tests/test_gpu.py tests/test_stream.py -m gpu -x -q --timeout 500 --timeout-method thread"
