# round 4: k_dp_spec_lean at 96 SGPRs (7 waves per SIMD, 4 spills: sg96) vs 80 (8 waves, 23 spills: base)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04an
mkdir -p $OUT
export TMPDIR=/tmp
for v in base sg96 base sg96; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --no-shapes --no-decode --cpu-seconds 0.2 >> $OUT/head_$v.json 2>> $OUT/head_$v.err || exit 1
done
echo done > $OUT/ok
