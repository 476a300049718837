set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/zuab
mkdir -p $OUT
A="--no-verify --no-decode --no-stream --no-shapes --cpu-seconds 0.2 --steps 1 --warmup 1 --workload zeros_urandom --mb 268"
SMALLZ4_AMD_LIB=$PWD/smallz4_amd/lib/libsmallz4_amd_r02k.so timeout -k 10 200 python -u bench.py $A > $OUT/r02k.json 2> $OUT/r02k.err || exit 1
timeout -k 10 200 python -u bench.py $A > $OUT/new.json 2> $OUT/new.err || exit 1
SZ4_NO_BIG=1 timeout -k 10 200 python -u bench.py $A > $OUT/nobig.json 2> $OUT/nobig.err || exit 1
echo ok > $OUT/ok
