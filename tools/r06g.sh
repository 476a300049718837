#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r06g
bash tools/gpu_steps.sh $O \
 "gen|300|python3 tools/prof_shape.py silesia --reps 1 && python3 tools/prof_shape.py text4m --reps 1 && python3 tools/prof_shape.py zu --reps 1" \
 "e8|120|python3 tools/prof_shape.py enwik8 --reps 5" \
 "sil|120|python3 tools/prof_shape.py silesia --reps 3" \
 "txt|120|python3 tools/prof_shape.py text4m --reps 3" \
 "zu|150|python3 tools/prof_shape.py zu --reps 2" \
 "unlz4_sil|150|python3 tools/prof_unlz4.py silesia" \
 "tests|600|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread"
