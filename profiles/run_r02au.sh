# round 2: parallel parse-boundary repair (k_dp_fix<true>) on top of the parallel walk repair -- parity subset, A/B vs HEAD on 64 KiB and 4 MiB blocks, parse segment size 8192 for 4 MiB blocks, 4 MiB kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02au
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_stream.py -x -v --timeout 170 --timeout-method thread -k "every_level or shapes or edge_sizes or other_block_sizes or silesia or structured or stream_multiblock or golden or run_across or chunk_boundaries or long_matches or zeros or greedy or lazy" > $OUT/tests.log 2>&1 || exit 1
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 5 --warmup 2"
L=$GRAFT_REPO_ROOT/smallz4_amd/lib
for rep in 1 2; do
  for v in old new; do
    if [ $v = new ]; then lib=$L/libsmallz4_amd.so; else lib=$L/libsmallz4_amd_$v.so; fi
    SMALLZ4_AMD_LIB=$lib timeout -k 10 120 python -u bench.py $A > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || exit 1
    SMALLZ4_AMD_LIB=$lib timeout -k 10 120 python -u bench.py $A --block-size 4194304 --mb 64 > $OUT/ab4m_${v}_$rep.json 2> $OUT/ab4m_${v}_$rep.err || exit 1
  done
  SZ4_DP_SIZE=8192 timeout -k 10 120 python -u bench.py $A --block-size 4194304 --mb 64 > $OUT/ab4m_dp8k_$rep.json 2> $OUT/ab4m_dp8k_$rep.err || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace4m -o bench -- \
  python3 $GRAFT_REPO_ROOT/bench.py $A --block-size 4194304 --mb 64 > $GRAFT_REPO_ROOT/$OUT/trace4m.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace64k -o bench -- \
  python3 $GRAFT_REPO_ROOT/bench.py $A > $GRAFT_REPO_ROOT/$OUT/trace64k.log 2>&1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
