# round 2: k_dp_spec_lean at 80 SGPRs (8 waves/SIMD instead of 6) -- parse parity subset, interleaved headline A/B vs HEAD (3 reps), lean kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 170 --timeout-method thread -k "every_level or shapes or long_matches or greedy or edge_sizes or other_block or structured or silesia or golden" > $OUT/tests.log 2>&1 || exit 1
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 10 --warmup 3"
L=$GRAFT_REPO_ROOT/smallz4_amd/lib
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = new ]; then lib=$L/libsmallz4_amd.so; else lib=$L/libsmallz4_amd_$v.so; fi
    SMALLZ4_AMD_LIB=$lib timeout -k 10 120 python -u bench.py $A > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || exit 1
  done
done
timeout -k 10 120 python -u bench.py $A --block-size 4194304 --mb 64 > $OUT/ab4m_new.json 2> $OUT/ab4m_new.err || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o bench -- \
  python3 $GRAFT_REPO_ROOT/bench.py $A > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
