# round 3: k_find_big phase costs on binary records (timing knobs; results wrong on purpose except dbg=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03d
mkdir -p $OUT
export TMPDIR=/tmp
for d in 0 1 2 3 7; do
SZ4_BIG_DBG=$d timeout -k 10 200 python -u profiles/probe_shapes.py --mb 48 --block-size 4194304 --kinds db > $OUT/db_dbg$d.jsonl 2>> $OUT/err.log || exit 1
done
timeout -k 10 200 python -u profiles/probe_shapes.py --mb 48 --block-size 4194304 --kinds text > $OUT/text.jsonl 2>> $OUT/err.log || exit 1
echo done > $OUT/ok
