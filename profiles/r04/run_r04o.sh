# round 4: parse fast batches v2 (packed lengths, keys shifted into rows) and the cheaper filter hit
# (base) vs the round-3 hit (hit1): compressor parity tests,
# headline bench; configs[4] kernel trace (where its parse time goes)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/test_gpu.log 2>&1 || exit 1
for v in base hit1; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $OUT/head_$v.json 2> $OUT/head_$v.err || exit 1
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/zu -o zu -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload zeros_urandom --steps 2 --warmup 1 --no-verify --no-decode --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $GRAFT_REPO_ROOT/$OUT/zu.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
