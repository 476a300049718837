# round 2 (re-entry): kernel profile of HEAD (trace + PMC passes), then the stream / shard / decoder suites
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02f
mkdir -p $OUT
bash profiles/collect.sh r02f &&
timeout -k 10 700 python -u -m pytest tests/test_stream.py tests/test_shards.py tests/test_unlz4.py -x -v --timeout 300 --timeout-method thread > $OUT/other_tests.log 2>&1
