# round 4, final tree: the whole GPU suite (per-test durations), then the profile collection
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ai
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread --durations=25 \
  > gpurun_out/r04ai/tests.log 2>&1 || exit 1
bash profiles/collect.sh r04ai
