# round 4: k_dp_fix converges at the first chunk of a segment whose positions down to its bottom all take
# one run's match unconditionally (base) vs walking them (ff0): parity tests, configs[4] A/B with its
# sampled diff against the reference, headline
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04ah
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu.py tests/test_shards.py tests/test_stream.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
for v in base ff0; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 400 python3 -u bench.py --workload zeros_urandom --steps 3 --warmup 1 --no-stream --no-dict --no-shapes --no-decode --verify-seconds 60 --cpu-seconds 0.2 > $OUT/zu_$v.json 2> $OUT/zu_$v.err || exit 1
done
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --no-shapes --no-decode --cpu-seconds 0.2 > $OUT/head.json 2> $OUT/head.err || exit 1
echo done > $OUT/ok
