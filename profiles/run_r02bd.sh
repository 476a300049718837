# round 2: final tree (lean parse at 80 SGPRs, no-match flag carried in the repair records) -- test_gpu.py + test_stream.py, then profiles/collect.sh (bench, kernel trace, PMC passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bd
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu.py tests/test_stream.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
bash profiles/collect.sh r02bd
