# round 4: configs[4] parse -- the parallel range-minimum repair threshold (SZ4_PAR_RMQ_MIN 64 / 16 / 8)
# and 4096-position parse segments for blocks above 64 KiB (SZ4_DP_SIZE), on a 300 MB zeros/urandom slice
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04c
mkdir -p $OUT
export TMPDIR=/tmp
A="--workload zeros_urandom --mb 300 --steps 3 --warmup 1 --no-stream --no-dict --no-shapes --no-decode --cpu-seconds 0.2 --verify-seconds 6"
for v in base pr16 pr8; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 240 python -u bench.py $A > $OUT/$v.json 2> $OUT/$v.err || exit 1
  SZ4_DP_SIZE=4096 SMALLZ4_AMD_LIB=$L timeout -k 10 240 python -u bench.py $A > $OUT/${v}_dp4k.json 2> $OUT/${v}_dp4k.err || exit 1
done
echo done > $OUT/ok
