# round 4: the decoder's size-word chain walked wave-uniform through scalar loads: decoder and stream
# tests, kernel trace of the headline round trip
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04aj
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_unlz4.py tests/test_stream.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $OUT/head.json 2> $OUT/head.err || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/tr -o tr -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-verify --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $GRAFT_REPO_ROOT/$OUT/tr.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
