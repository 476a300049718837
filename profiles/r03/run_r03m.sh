# round 3: kernel split on db and the Silesia shape (4 MiB blocks)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03m
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for k in db silesia; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/$k -o t -- python3 $GRAFT_REPO_ROOT/profiles/probe_shapes.py --mb 32 --block-size 4194304 --kinds $k > $GRAFT_REPO_ROOT/$OUT/$k.log 2>&1 || exit 1
done
echo done > $GRAFT_REPO_ROOT/$OUT/ok
