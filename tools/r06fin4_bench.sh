#!/bin/bash
# the round's final bench line (default legs), into gpurun_out/r06fin4/ for profiles/summarize.py
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/r06fin4
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python3 "$R/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err"
