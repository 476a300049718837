# round 3: k_find_sorted_hbm with the text in HBM/L2 (no LDS window, 80 SGPRs: two workgroups per CU)
# against the LDS window; dictionary -6 kernel split
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03aa
mkdir -p $OUT
export TMPDIR=/tmp
A="--no-verify --no-decode --no-stream --no-shapes --cpu-seconds 0.2 --steps 3 --warmup 1"
for v in base hg; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python -u bench.py $A --block-size 4194304 > $OUT/t4m_$v.json 2> $OUT/t4m_$v.err || exit 1
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python -u bench.py $A --workload silesia > $OUT/sil_$v.json 2> $OUT/sil_$v.err || exit 1
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python -u bench.py $A --workload zeros_urandom --mb 268.435456 > $OUT/zu_$v.json 2> $OUT/zu_$v.err || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/dict -o t -- python3 $GRAFT_REPO_ROOT/tools/time_dict.py 8 > $GRAFT_REPO_ROOT/$OUT/dict.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
