# round 2: profile of HEAD (parallel parse/walk repair) -- smoke, bench, kernel trace and PMC passes (profiles/collect.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02av
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02av/smoke.log 2>&1 || exit 1
bash profiles/collect.sh r02av
