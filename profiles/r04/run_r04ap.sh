# round 4: two candidates per filter test in the below-chunk loop (fu1) vs one (base), k_find_sorted at two workgroups per CU
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04ap
mkdir -p $OUT
export TMPDIR=/tmp
for v in base fu1 base fu1; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --no-shapes --no-decode --cpu-seconds 0.2 >> $OUT/head_$v.json 2>> $OUT/head_$v.err || exit 1
done
echo done > $OUT/ok
