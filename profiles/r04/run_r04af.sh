# round 4: kernel traces of the 4 MiB-block shapes (text, Silesia mix); k_walk with the next window's
# tables built during the lifting (base) vs after it (wp0): compressor parity tests, headline A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04af
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/test_gpu.log 2>&1 || exit 1
for v in base wp0 base wp0; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --no-shapes --no-decode --cpu-seconds 0.2 >> $OUT/head_$v.json 2>> $OUT/head_$v.err || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/t4 -o t4 -- \
  python3 $GRAFT_REPO_ROOT/bench.py --block-size 4194304 --steps 3 --warmup 1 --no-verify --no-decode --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $GRAFT_REPO_ROOT/$OUT/t4.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/si -o si -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload silesia --steps 3 --warmup 1 --no-verify --no-decode --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $GRAFT_REPO_ROOT/$OUT/si.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
