# round 2: k_find_sorted few-targets path (lanes = candidates for a group's tail) -- A/B of the threshold, diag counters, parity
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02p
mkdir -p $OUT
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 10 --warmup 3"
L=$GRAFT_REPO_ROOT/smallz4_amd/lib
for rep in 1 2; do
  for v in few0 few12 default few40; do
    if [ $v = default ]; then lib=$L/libsmallz4_amd.so; else lib=$L/libsmallz4_amd_$v.so; fi
    SMALLZ4_AMD_LIB=$lib timeout -k 10 120 python -u bench.py $A > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || exit 1
  done
done
timeout -k 10 200 python -u tools/diag_find.py 100 > $OUT/diag.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 170 --timeout-method thread -k "every_level or shapes or long_matches or other_block_sizes or edge or finder_intermediate or structured or silesia or large_roundtrip" > $OUT/tests.log 2>&1
