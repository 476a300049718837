# round 2, first GPU pass: the new stream / shard tests, then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02a
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests/test_stream.py tests/test_shards.py -x -v --timeout 600 --timeout-method thread > $OUT/new_tests.log 2>&1 &&
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
