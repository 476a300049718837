# round 2: decoder with a 16 KiB LDS ring (far match bytes from drained output) -- decoder GPU tests, A/B of the device round trip vs HEAD, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02aw
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_unlz4.py -m gpu -x -v --timeout 170 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
A="--no-verify --no-stream --cpu-seconds 0.2 --steps 5 --warmup 2"
L=$GRAFT_REPO_ROOT/smallz4_amd/lib
for rep in 1 2; do
  for v in old new; do
    if [ $v = new ]; then lib=$L/libsmallz4_amd.so; else lib=$L/libsmallz4_amd_$v.so; fi
    SMALLZ4_AMD_LIB=$lib timeout -k 10 120 python -u bench.py $A > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || exit 1
  done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o bench -- \
  python3 $GRAFT_REPO_ROOT/bench.py $A > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
