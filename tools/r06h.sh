#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r06h
bash tools/gpu_steps.sh $O \
 "gen|300|python3 tools/prof_shape.py silesia --reps 1 && python3 tools/prof_shape.py zu --reps 1" \
 "zu|150|python3 tools/prof_shape.py zu --reps 2" \
 "e8|120|python3 tools/prof_shape.py enwik8 --reps 5" \
 "sil|120|python3 tools/prof_shape.py silesia --reps 3" \
 "diagzu|200|python3 tools/diag_find.py 268 65535 zu" \
 "tests|400|python -u -m pytest tests/test_gpu.py tests/test_shards.py -m gpu -x -q --timeout 300 --timeout-method thread"
