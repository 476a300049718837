# round 3: run-aware k_find_big -- parity on the block fixtures and structured content, then the Silesia shape
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 170 --timeout-method thread -k "golden_fixtures or structured or silesia or long_matches or shapes or every_level or finder or long_run" > $OUT/tests.log 2>&1 || exit 1
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 3 --warmup 1"
timeout -k 10 200 python -u bench.py $A --workload silesia > $OUT/silesia.json 2> $OUT/silesia.err || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/silesia_trace -o t -- python3 $GRAFT_REPO_ROOT/bench.py $A --workload silesia > $GRAFT_REPO_ROOT/$OUT/silesia_trace.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
