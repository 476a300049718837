set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r01i
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01i/gpu_tests.log 2>&1
