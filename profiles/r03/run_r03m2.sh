# round 3: bisect the slow 256 MiB piece of configs[4]'s slice (256..512 MiB) in 16 MiB, then 1 MiB pieces
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03m2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/zu_pieces.py 16 512 256 > $OUT/p16.jsonl 2> $OUT/p16.err || exit 1
echo done > $OUT/ok
