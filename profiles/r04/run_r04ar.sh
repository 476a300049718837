# round 4, exact final tree (k_find_long9 repair early exit included): the whole GPU suite, smoke(), then the profile collection
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04ar
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread --durations=10 \
  > gpurun_out/r04ar/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04ar/smoke.log 2>&1 || exit 1
bash profiles/collect.sh r04ar
