# round 4: __graft_entry__.smoke() and the default bench line on the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04ag
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done > $OUT/ok
