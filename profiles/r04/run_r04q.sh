# round 4: decoder sizes pass on the vector unit (token chain by binary lifting per 64 window
# positions) vs the one-sequence-at-a-time walk (unser): decoder parity tests, headline bench with its
# device round trip, kernel trace of the headline round trip
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_unlz4.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/test_unlz4.log 2>&1 || exit 1
for v in base unser; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $OUT/head_$v.json 2> $OUT/head_$v.err || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/tr -o tr -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-verify --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $GRAFT_REPO_ROOT/$OUT/tr.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
