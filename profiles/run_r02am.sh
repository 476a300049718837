# round 2: k_find_sorted occupancy / stall counters (one SQ pass + GRBM clock), counter list
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r02am
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
ARGS="--steps 3 --warmup 1 --no-verify --no-decode --no-stream --cpu-seconds 0.2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT \
  --kernel-include-regex k_find_sorted --output-format csv -d $OUT/sqA -o bench -- python3 $R/bench.py $ARGS > $OUT/sqA.log 2>&1
