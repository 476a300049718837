# round 4: the whole GPU suite (per-test durations) and the profile collection on the current tree
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04n
export TMPDIR=/tmp
timeout -k 10 800 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread --durations=40 \
  > gpurun_out/r04n/tests.log 2>&1 || exit 1
bash profiles/collect.sh r04n
