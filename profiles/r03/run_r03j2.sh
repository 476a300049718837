# round 3: XCD-aware segment order in k_find_sorted_hbm (each XCD a contiguous run of segments, so the
# shared windows stay in its L2) vs blockIdx order; parity of 4 MiB / 256 KiB block shapes; FETCH pass
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03j2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "silesia or structured or block_sizes or stream_multiblock or zero" > $OUT/tests.log 2>&1 || exit 1
A="--no-verify --no-decode --no-stream --no-shapes --cpu-seconds 0.2 --steps 3 --warmup 1"
for v in xcd noxcd; do
  if [ $v = xcd ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python -u bench.py $A --workload silesia > $OUT/sil_$v.json 2> $OUT/sil_$v.err || exit 1
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python -u bench.py $A --block-size 4194304 > $OUT/t4m_$v.json 2> $OUT/t4m_$v.err || exit 1
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python -u bench.py $A --workload zeros_urandom --mb 268.435456 > $OUT/zu_$v.json 2> $OUT/zu_$v.err || exit 1
done
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$OUT/fetch -o t -- python3 $GRAFT_REPO_ROOT/bench.py $A --block-size 4194304 > $GRAFT_REPO_ROOT/$OUT/fetch.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
