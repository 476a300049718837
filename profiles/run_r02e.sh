# round 2 (re-entry): HEAD on the GPU -- bench line first, then the core parity suite
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02e
mkdir -p $OUT
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 840 python -u -m pytest tests/test_gpu.py -x -v --timeout 170 --timeout-method thread > $OUT/gpu_tests.log 2>&1
