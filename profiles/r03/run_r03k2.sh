# round 3: which kernel makes configs[4]'s 1.25 GiB slice slow (pieces 2-4 each hold a zero run longer
# than a 256 KiB block); per block layout, with a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03k2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/zu_block_kinds.py > $OUT/kinds.jsonl 2> $OUT/kinds.err || exit 1
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/whole -o t -- python3 $GRAFT_REPO_ROOT/tools/zu_block_kinds.py whole > $GRAFT_REPO_ROOT/$OUT/whole.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
