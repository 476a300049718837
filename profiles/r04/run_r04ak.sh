# round 4: the parse's fast-chunk test by one ballot (every length <= 64) instead of a row reduction:
# compressor parity tests, headline x2
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04ak
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/test_gpu.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --no-shapes --no-decode --cpu-seconds 0.2 >> $OUT/head.json 2>> $OUT/head.err || exit 1
done
echo done > $OUT/ok
