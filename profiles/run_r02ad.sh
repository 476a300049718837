# round 2: k_find_sorted: below-chunk prefetch issued with the chunk slots -- A/B, parity
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02ad
mkdir -p $OUT
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 10 --warmup 3"
L=$GRAFT_REPO_ROOT/smallz4_amd/lib
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = new ]; then lib=$L/libsmallz4_amd.so; else lib=$L/libsmallz4_amd_$v.so; fi
    SMALLZ4_AMD_LIB=$lib timeout -k 10 120 python -u bench.py $A > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || exit 1
  done
done
for v in old new; do
  if [ $v = new ]; then lib=$L/libsmallz4_amd.so; else lib=$L/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$lib timeout -k 10 120 python -u bench.py $A --level 3 > $OUT/l3_${v}.json 2> $OUT/l3_${v}.err || exit 1
done
timeout -k 10 700 python -u -m pytest tests/test_gpu.py -x -v --timeout 170 --timeout-method thread -k "every_level or shapes or long_matches or other_block_sizes or edge or structured or greedy_lazy or finder_intermediate or large_roundtrip" > $OUT/tests.log 2>&1
