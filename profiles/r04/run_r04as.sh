# round 4: k_write_seg launch bound for 7 (ww7: 72 VGPRs, 3 spilled) or 8 (ww8: 64, 12 spilled) waves per SIMD vs none (base: 77, 6 waves)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04as
mkdir -p $OUT
export TMPDIR=/tmp
for v in base ww7 ww8 base ww7 ww8; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --no-shapes --no-decode --cpu-seconds 0.2 >> $OUT/head_$v.json 2>> $OUT/head_$v.err || exit 1
done
echo done > $OUT/ok
