# round 2: stream/shard suites on the current tree, then the other shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02s
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests/test_stream.py tests/test_shards.py -x -v --timeout 400 --timeout-method thread > $OUT/stream_shard_tests.log 2>&1 &&
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 3 --warmup 1"
for L in 1 2 3 6; do
  timeout -k 10 200 python -u bench.py $A --level $L > $OUT/enwik8_l$L.json 2> $OUT/enwik8_l$L.err || exit 1
done
for w in silesia zeros_urandom random zeros; do
  timeout -k 10 300 python -u bench.py $A --workload $w > $OUT/$w.json 2> $OUT/$w.err || exit 1
done
timeout -k 10 200 python -u bench.py $A --workload enwik8 --block-size 4194304 --mb 64 > $OUT/enwik8_4m.json 2> $OUT/enwik8_4m.err
