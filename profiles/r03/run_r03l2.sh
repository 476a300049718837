# round 3: configs[4]'s 1.25 GiB rank slice piece by piece (which 256 MiB piece makes find_long slow)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03l2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/zu_pieces.py 256 1280 > $OUT/pieces.jsonl 2> $OUT/pieces.err || exit 1
echo done > $OUT/ok
