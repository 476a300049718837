# round 4: assemble latency (k_walk four windows in flight, k_seg_tokens loads two batches ahead,
# k_write_seg literal runs 8 bytes per load round) + the parse's reach scan prefetch (base) vs the
# previous tree (prev), plus the in-vector literal bump in the parse's fast chunks: compressor parity tests,
# headline A/B, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/test_gpu.log 2>&1 || exit 1
for v in base prev base prev; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --no-shapes --no-decode --cpu-seconds 0.2 >> $OUT/head_$v.json 2>> $OUT/head_$v.err || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/tr -o tr -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-verify --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $GRAFT_REPO_ROOT/$OUT/tr.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
