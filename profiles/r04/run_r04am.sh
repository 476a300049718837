# round 4: in-chunk candidates of one-first-word chunks by broadcast (base) vs through the shift register
# (ss0): compressor parity tests, headline A/B x2, shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04am
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/test_gpu.log 2>&1 || exit 1
for v in base ss0 base ss0; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --no-shapes --no-decode --cpu-seconds 0.2 >> $OUT/head_$v.json 2>> $OUT/head_$v.err || exit 1
done
timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --no-stream --no-dict --cpu-seconds 0.2 > $OUT/shapes.json 2> $OUT/shapes.err || exit 1
echo done > $OUT/ok
