# round 3: hybrid class path (by group size) A/B + run hand-off threshold; parity first
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03t
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "golden or structured or silesia" > $OUT/tests.log 2>&1 || exit 1
for v in base cw1k cw16k cwinf rl2048; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 200 python -u profiles/probe_shapes.py --mb 32 --block-size 4194304 --kinds text,xml,exe,db,src,silesia > $OUT/$v.jsonl 2> $OUT/$v.err || exit 1
  SMALLZ4_AMD_LIB=$L timeout -k 10 200 python -u profiles/probe_shapes.py --mb 64 --block-size 262144 --kinds zu >> $OUT/$v.jsonl 2>> $OUT/$v.err || exit 1
done
echo done > $OUT/ok
