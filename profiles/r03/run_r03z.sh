# round 3: LPF targets need 12-byte agreement among the probes (ll2/ll4), run-key hand-off threshold (rl);
# dictionary -6 after the skip-kernel fix
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03z
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/time_dict.py 8 > $OUT/dict.jsonl 2> $OUT/dict.err || exit 1
for v in base ll2 ll4 rl ll2rl; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 200 python -u profiles/probe_shapes.py --mb 32 --block-size 4194304 --kinds text,xml,exe,db,src,silesia > $OUT/$v.jsonl 2> $OUT/$v.err || exit 1
done
echo done > $OUT/ok
