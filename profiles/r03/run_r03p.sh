# round 3: full GPU suite + default bench (shapes leg, verify) + stream leg
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done > $OUT/ok
