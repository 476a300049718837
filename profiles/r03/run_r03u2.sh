# round 3 final tree: the driver's smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03u2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03u2/smoke.log 2>&1 || exit 1
