# round 2 (re-entry): the whole GPU suite on HEAD, then the profile (trace + PMC) of the bench workload
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02as
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 450 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
bash profiles/collect.sh r02as
