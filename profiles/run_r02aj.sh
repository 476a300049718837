# round 2: k_find_sorted phase-skip timing (results deliberately wrong in the x* variants; --no-verify)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02aj
mkdir -p $OUT
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 5 --warmup 2"
L=$GRAFT_REPO_ROOT/smallz4_amd/lib
for v in new old xnofilt xshift xbcast xboth; do
  if [ $v = new ]; then lib=$L/libsmallz4_amd.so; else lib=$L/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$lib timeout -k 10 120 python -u bench.py $A > $OUT/ab_${v}.json 2> $OUT/ab_${v}.err || exit 1
done
