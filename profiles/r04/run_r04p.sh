# round 4: parse repair (k_dp_fix) reads a same-letter run's end once per run and prefetches two
# chunks ahead; k_dp_spec reads the run end once per run: compressor + stream parity tests, headline
# bench, configs[4] kernel trace and bench line with its sampled diff
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04p
mkdir -p $OUT
export TMPDIR=/tmp
# (first pass: tools/bin/valu_ceiling, test_gpu + test_stream 153 passed; test_shards re-run alone)
timeout -k 10 900 python3 -u -m pytest tests/test_shards.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests_shards.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $OUT/head.json 2> $OUT/head.err || exit 1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/zu -o zu -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload zeros_urandom --steps 2 --warmup 1 --no-verify --no-decode --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $GRAFT_REPO_ROOT/$OUT/zu.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
