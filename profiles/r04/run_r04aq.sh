# round 4: k_write_seg staging each 64-token chunk in LDS, copied out as aligned dwords (base) vs direct byte stores (ws0, the committed tree)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04aq
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
for v in base ws0 base ws0; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --no-shapes --no-decode --cpu-seconds 0.2 >> $OUT/head_$v.json 2>> $OUT/head_$v.err || exit 1
done
echo done > $OUT/ok
