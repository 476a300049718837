# round 2: sizes pass on block-relative cursors without bounds checks (last 20 bytes byte-wise) -- decoder GPU tests, A/B vs the previous commit, kernel trace; then the other shapes on the current tree
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02ax
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
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 3 --warmup 1"
for L in 1 2 3 6; do
  timeout -k 10 200 python -u bench.py $A --level $L > $OUT/enwik8_l$L.json 2> $OUT/enwik8_l$L.err || exit 1
done
for w in silesia zeros_urandom random; do
  timeout -k 10 300 python -u bench.py $A --workload $w > $OUT/$w.json 2> $OUT/$w.err || exit 1
done
timeout -k 10 200 python -u bench.py $A --workload enwik8 --block-size 4194304 --mb 64 > $OUT/enwik8_4m.json 2> $OUT/enwik8_4m.err || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o bench -- \
  python3 $GRAFT_REPO_ROOT/bench.py --no-verify --no-stream --cpu-seconds 0.2 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
