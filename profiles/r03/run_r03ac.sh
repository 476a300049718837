# round 3: LPF thresholds again on the HBM/L2 text path; the drop-in stream path timed in C++ (1 GB)
# and its kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03ac
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 bash tools/stream_big.sh $OUT 10 > $OUT/stream.log 2>&1 || exit 1
for v in base ll2 lpf1k lpf8k; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 200 python -u profiles/probe_shapes.py --mb 32 --block-size 4194304 --kinds text,xml,exe,db,src,silesia > $OUT/$v.jsonl 2> $OUT/$v.err || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/stream_trace -o t -- $GRAFT_REPO_ROOT/tools/bin/stream_threads big 9 /tmp/sz4_stream_base.bin 3 /dev/null > $GRAFT_REPO_ROOT/$OUT/stream_trace.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
