# round 3: stream path (download overlapped with the next read, warm first call), test_stream.py whole
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03ae
mkdir -p $OUT
export TMPDIR=/tmp
SZ4_STREAM_PROFILE=1 timeout -k 10 400 bash tools/stream_big.sh $OUT 10 > $OUT/stream.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_stream.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests_stream.log 2>&1 || exit 1
echo done > $OUT/ok
