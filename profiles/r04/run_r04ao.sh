# round 4: k_find_long9's repair launches leave before staging the window when no piece head needs a
# walk: compressor + stream parity tests, headline x2, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04ao
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py tests/test_stream.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --no-shapes --no-decode --cpu-seconds 0.2 >> $OUT/head.json 2>> $OUT/head.err || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/tr -o tr -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-verify --no-decode --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $GRAFT_REPO_ROOT/$OUT/tr.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
