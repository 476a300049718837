# round 2: the rest of the stream / shard tests; level 1-6 bench lines (parallel greedy/lazy replay)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02c
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_stream.py tests/test_shards.py -x -v --timeout 170 --timeout-method thread -k "not golden and not boundaries" > $OUT/new_tests.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 170 --timeout-method thread -k "every_level or greedy_lazy or golden or edge_sizes or shapes or intermediate or stream_multiblock" > $OUT/lazy_tests.log 2>&1 &&
for L in 1 2 3 6; do timeout -k 10 200 python -u bench.py --level $L --steps 5 --warmup 2 --no-stream --no-decode --cpu-seconds 1 --verify-blocks 64 > $OUT/bench_l$L.json 2> $OUT/bench_l$L.err || exit 1; done
