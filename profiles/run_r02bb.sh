# round 2: final tree -- interleaved headline A/B (fence-only parse repair vs + no-match segments), then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bb
mkdir -p $OUT
export TMPDIR=/tmp
A="--no-verify --no-stream --cpu-seconds 0.2 --steps 10 --warmup 3"
L=$GRAFT_REPO_ROOT/smallz4_amd/lib
for rep in 1 2; do
  for v in old new; do
    if [ $v = new ]; then lib=$L/libsmallz4_amd.so; else lib=$L/libsmallz4_amd_$v.so; fi
    SMALLZ4_AMD_LIB=$lib timeout -k 10 120 python -u bench.py $A > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || exit 1
  done
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || exit 1
echo done > $OUT/ok
