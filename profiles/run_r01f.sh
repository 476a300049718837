set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r01f
timeout -k 10 400 python -u -m pytest tests/test_unlz4.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r01f/unlz4_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r01f/bench.json 2> gpurun_out/r01f/bench.err && \
SZ4_SEPARATE_SORT=1 timeout -k 10 300 python bench.py --no-verify --no-decode --cpu-seconds 0.5 > gpurun_out/r01f/bench_separate_sort.json 2>> gpurun_out/r01f/bench.err && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r01f/smoke.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_unlz4.py > gpurun_out/r01f/gpu_tests.log 2>&1
