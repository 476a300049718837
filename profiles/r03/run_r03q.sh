# round 3 final tree (walk table, run-key sampling), part 1: the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1150 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
echo done > $OUT/tests_ok
