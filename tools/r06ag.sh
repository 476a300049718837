#!/bin/bash
O=gpurun_out/r06ag
bash tools/gpu_steps.sh $O \
 "sil|300|python3 tools/diag_unlz4.py silesia" \
 "txt|300|python3 tools/diag_unlz4.py text4m"
