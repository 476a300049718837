# round 2: k_find_long9_lds at 80 SGPRs (two workgroups per CU) -- pass-2 parity subset, interleaved headline A/B vs the lean-parse tree (3 reps)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02be
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 170 --timeout-method thread -k "every_level or shapes or long_matches or edge_sizes or other_block or structured or silesia or finder or long_run" > $OUT/tests.log 2>&1 || exit 1
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 10 --warmup 3"
L=$GRAFT_REPO_ROOT/smallz4_amd/lib
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = new ]; then lib=$L/libsmallz4_amd.so; else lib=$L/libsmallz4_amd_$v.so; fi
    SMALLZ4_AMD_LIB=$lib timeout -k 10 120 python -u bench.py $A > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || exit 1
  done
done
echo done > $OUT/ok
