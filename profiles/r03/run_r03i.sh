# round 3: token walk with a per-window next-match table (two readlanes per step) vs the ballot walk;
# parity of the emitted frames
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "golden or level or blocks or edge or stream_multiblock" > $OUT/tests.log 2>&1 || exit 1
A="--no-verify --no-decode --no-stream --no-shapes --cpu-seconds 0.2 --steps 20 --warmup 3"
for i in 1 2 3; do
  for v in new old; do
    if [ $v = new ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_oldwalk.so; fi
    SMALLZ4_AMD_LIB=$L timeout -k 10 200 python -u bench.py $A > $OUT/ab_${v}_$i.json 2> $OUT/ab_${v}_$i.err || exit 1
  done
done
echo done > $OUT/ok
