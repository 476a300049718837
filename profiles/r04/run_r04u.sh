# round 4: the whole GPU suite on the current tree (per-test durations), then the profile collection
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04u
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread --durations=25 \
  > gpurun_out/r04u/tests.log 2>&1 || exit 1
bash profiles/collect.sh r04u
