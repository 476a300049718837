# round 3: the slow block(s) of configs[4]'s slice between 304 and 320 MiB, one block per call
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03n2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/zu_blocks.py 304 64 > $OUT/blocks.jsonl 2> $OUT/blocks.err || exit 1
echo done > $OUT/ok
