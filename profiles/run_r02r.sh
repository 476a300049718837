# round 2: decoder as sequence list + replay -- decoder parity suite, the two-rank bench test, the bench's device round trip, trace
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02r
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_unlz4.py -x -v --timeout 170 --timeout-method thread > $OUT/unlz4_tests.log 2>&1 &&
timeout -k 10 500 python -u -m pytest tests/test_shards.py -x -v --timeout 450 --timeout-method thread -k two_ranks > $OUT/two_ranks.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-stream --cpu-seconds 0.5 --verify-blocks 64 > $OUT/bench.json 2> $OUT/bench.err &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o t -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-verify --no-stream --cpu-seconds 0.2 > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1
