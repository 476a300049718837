#!/bin/bash
# Round-N profile collection on the MI355X box (run from the repo root through gpurun):
#   bash profiles/collect.sh rNN [bench.py workload args, e.g. --workload silesia]
# Writes gpurun_out/<tag>/: the bench JSON line, a rocprofv3 kernel-trace --stats summary of the
# same workload, and separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ issue counters + GRBM_GUI_ACTIVE for
# the clock).  SKIP_BENCH=1 leaves out the full bench line (profile only).  Each GPU
# step has its own time limit and the chain stops at the first failure.
set -euo pipefail
TAG=${1:-r01}
shift || true
EXTRA="$*"
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "${SKIP_BENCH:-}" ]; then
  timeout -k 10 700 python3 "$R/bench.py" $EXTRA > "$OUT/bench.json" 2> "$OUT/bench.err"
fi
cd /tmp
ARGS="--steps 10 --warmup 3 --no-verify --no-stream --no-dict --no-shapes --no-levels --cpu-seconds 0.5 $EXTRA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
  python3 "$R/bench.py" $ARGS > "$OUT/trace.log" 2>&1
ARGS="--steps 3 --warmup 1 --no-verify --no-decode --no-stream --no-dict --no-shapes --no-levels --cpu-seconds 0.5 $EXTRA"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o bench -- \
  python3 "$R/bench.py" $ARGS > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o bench -- \
  python3 "$R/bench.py" $ARGS > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/sq" -o bench -- python3 "$R/bench.py" $ARGS > "$OUT/sq.log" 2>&1
echo done > "$OUT/ok"
