# round 3: where the drop-in stream path's time goes (callbacks vs GPU); LPF class-dominance slack A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03ad
mkdir -p $OUT
export TMPDIR=/tmp
SZ4_STREAM_PROFILE=1 timeout -k 10 400 bash tools/stream_big.sh $OUT 10 > $OUT/stream.log 2>&1 || exit 1
for v in base s1 s0; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 200 python -u profiles/probe_shapes.py --mb 32 --block-size 4194304 --kinds text,xml,exe,db,src,silesia > $OUT/$v.jsonl 2> $OUT/$v.err || exit 1
done
echo done > $OUT/ok
