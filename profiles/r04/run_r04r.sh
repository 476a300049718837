# round 4: block decode 64 output bytes per step (sequence map by LDS marks + max-scan, in-window match
# bytes by pointer jumping) vs one sequence per step (decser): decoder and stream parity tests, headline bench with its
# device round trip, kernel trace of the headline round trip
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_unlz4.py tests/test_stream.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/test_unlz4.log 2>&1 || exit 1
for v in base decser; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $OUT/head_$v.json 2> $OUT/head_$v.err || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/tr -o tr -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-verify --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $GRAFT_REPO_ROOT/$OUT/tr.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
