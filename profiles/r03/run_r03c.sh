# round 3: per-kind stage times at 4 MiB blocks (48 MB per kind) and kernel traces of db and xml
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u profiles/probe_shapes.py --mb 48 --block-size 4194304 --kinds text,xml,exe,db,image,src > $OUT/kinds_4m.jsonl 2> $OUT/kinds.err || exit 1
cd /tmp
for k in db xml exe; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_$k -o t -- python3 $GRAFT_REPO_ROOT/profiles/probe_shapes.py --mb 48 --block-size 4194304 --kinds $k > $GRAFT_REPO_ROOT/$OUT/trace_$k.log 2>&1 || exit 1
done
echo done > $GRAFT_REPO_ROOT/$OUT/ok
