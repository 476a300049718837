# round 4: dictionary leg A/B -- the 1-hop run skip in k_dict_search (base) vs without (variant norunskip)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04f
mkdir -p $OUT
export TMPDIR=/tmp
A="--mb 1 --steps 1 --warmup 1 --no-stream --no-shapes --no-decode --no-verify --cpu-seconds 0.1"
timeout -k 10 300 python -u bench.py $A > $OUT/base.json 2> $OUT/base.err || exit 1
SMALLZ4_AMD_LIB=smallz4_amd/lib/libsmallz4_amd_norunskip.so timeout -k 10 300 python -u bench.py $A > $OUT/norunskip.json 2> $OUT/norunskip.err || exit 1
echo done > $OUT/ok
