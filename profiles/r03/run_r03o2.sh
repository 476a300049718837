# round 3: the slow configs[4] block -- kernel trace and k_find_big's phase counters
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03o2
mkdir -p $OUT
export TMPDIR=/tmp
SMALLZ4_AMD_LIB=$GRAFT_REPO_ROOT/smallz4_amd/lib/libsmallz4_amd_diag.so timeout -k 10 200 python -u tools/zu_slow.py > $OUT/diag.jsonl 2> $OUT/diag.err || exit 1
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o t -- python3 $GRAFT_REPO_ROOT/tools/zu_slow.py > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
