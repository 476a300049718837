# round 4, exact final tree: the whole GPU suite and smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04al
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread --durations=10 \
  > gpurun_out/r04al/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04al/smoke.log 2>&1 || exit 1
