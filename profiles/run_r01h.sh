set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r01h_smoke.log 2>&1 && bash profiles/collect.sh r01h
