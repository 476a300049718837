# round 2: final tree (pass 2 at 80 SGPRs) -- the GPU tests r02be's subset left out: the rest of test_gpu.py, test_stream.py, test_shards.py, test_unlz4.py
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bf
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 840 python -u -m pytest tests/test_gpu.py tests/test_stream.py tests/test_shards.py tests/test_unlz4.py -m gpu -x -v --timeout 200 --timeout-method thread -k "not (every_level or shapes or long_matches or edge_sizes or other_block or structured or silesia or finder or long_run)" > $OUT/tests.log 2>&1 || exit 1
echo done > $OUT/ok
