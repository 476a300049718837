#!/bin/bash
O=gpurun_out/r06ar
bash tools/gpu_steps.sh $O \
 "suite|1000|python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread"
