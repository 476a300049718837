# round 4: row-transposed parse batches and the vector forward walk (the product lib) vs the scalar parse batches (dpold) and the scalar walk (walkold):
# the GPU parity tests of the compressor, then the headline bench (every block diffed against the
# reference) for both, then the shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread --durations=20 > $OUT/test_gpu.log 2>&1 || exit 1
for v in base dpold walkold; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $OUT/head_$v.json 2> $OUT/head_$v.err || exit 1
done
timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --no-stream --no-dict --cpu-seconds 0.2 > $OUT/shapes.json 2> $OUT/shapes.err || exit 1
echo done > $OUT/ok
