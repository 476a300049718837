# round 3: A/B of the find_big hand-off thresholds (run keys, LPF) at 4 MiB blocks
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03r
mkdir -p $OUT
export TMPDIR=/tmp
for v in base rl256 rl2048 lpf1k nolpf; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 200 python -u profiles/probe_shapes.py --mb 32 --block-size 4194304 --kinds text,xml,exe,db,src,silesia > $OUT/$v.jsonl 2> $OUT/$v.err || exit 1
done
echo done > $OUT/ok
