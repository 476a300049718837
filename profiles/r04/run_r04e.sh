# round 4: k_find_sorted A/B on the headline workload -- MSD sort fused (base), the round-3 LSD sort
# (variant lsd), separate k_sort launch, text from HBM/L2 instead of the LDS window (k_find_sorted_hbm on
# 64 KiB blocks)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04e
mkdir -p $OUT
export TMPDIR=/tmp
A="--steps 10 --warmup 3 --no-stream --no-dict --no-shapes --no-decode --no-verify --cpu-seconds 0.2"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --no-shapes --no-decode --cpu-seconds 0.2 > $OUT/base.json 2> $OUT/base.err || exit 1
SMALLZ4_AMD_LIB=smallz4_amd/lib/libsmallz4_amd_lsd.so timeout -k 10 240 python -u bench.py $A > $OUT/lsd.json 2> $OUT/lsd.err || exit 1
SZ4_SEPARATE_SORT=1 timeout -k 10 240 python -u bench.py $A > $OUT/sep.json 2> $OUT/sep.err || exit 1
SZ4_FIND_HBM=1 timeout -k 10 240 python -u bench.py $A > $OUT/hbm.json 2> $OUT/hbm.err || exit 1
echo done > $OUT/ok
