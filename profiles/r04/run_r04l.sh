# round 4: the whole GPU suite on the current tree, with per-test durations
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04l
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread --durations=60 \
  > gpurun_out/r04l/tests.log 2>&1
