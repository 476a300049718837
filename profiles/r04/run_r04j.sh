# round 4: LPF routing decided from the chunk (variant lpfl) vs the 8-probe decision, on configs[2]
# (Silesia-shaped, 4 MiB blocks) and text at 4 MiB blocks; sampled byte diff against the reference
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04j
mkdir -p $OUT
export TMPDIR=/tmp
for v in base lpfl; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 400 python -u bench.py --workload silesia --steps 3 --warmup 1 --no-stream --no-dict --no-shapes --verify-seconds 20 --cpu-seconds 0.2 > $OUT/sil_$v.json 2> $OUT/sil_$v.err || exit 1
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python -u bench.py --block-size 4194304 --steps 3 --warmup 1 --no-stream --no-dict --no-shapes --no-verify --cpu-seconds 0.2 > $OUT/t4m_$v.json 2> $OUT/t4m_$v.err || exit 1
done
echo done > $OUT/ok
