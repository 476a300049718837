# round 3: the whole GPU suite on the new tree (run table, pipelined stream path, pieced batch API), then perf
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u profiles/probe_shapes.py --mb 48 --block-size 4194304 --kinds text,xml,exe,db,image,src > $OUT/kinds_4m.jsonl 2> $OUT/kinds.err || exit 1
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done > $OUT/ok
