# round 2: LDS-tiled sort + text-order result tiles in k_find_sorted; stream/shard tests; bench
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02b
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v --timeout 170 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-stream --cpu-seconds 2 > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 900 python -u -m pytest tests/test_stream.py tests/test_shards.py -x -v --timeout 170 --timeout-method thread > $OUT/new_tests.log 2>&1
