# round 2: unrolled fast batches in k_dp_spec -- bench first, then the whole test_gpu suite
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02m
mkdir -p $OUT
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-stream --cpu-seconds 1 > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v --timeout 170 --timeout-method thread > $OUT/gpu_tests.log 2>&1
