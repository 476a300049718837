#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r06k
bash tools/gpu_steps.sh $O \
 "gen|300|python3 tools/prof_shape.py silesia --reps 1 && python3 tools/prof_shape.py zu --reps 1" \
 "zu|150|python3 tools/prof_shape.py zu --reps 2" \
 "sil|120|python3 tools/prof_shape.py silesia --reps 3" \
 "e8|120|python3 tools/prof_shape.py enwik8 --reps 5" \
 "bigzu|200|python3 tools/diag_big.py 268 zu" \
 "tests|500|python -u -m pytest tests/test_gpu.py tests/test_shards.py tests/test_stream.py -m gpu -x -q --timeout 300 --timeout-method thread"
