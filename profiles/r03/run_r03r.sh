# round 3 final tree, part 2: profile collections for the headline workload (r03r) and the Silesia shape (r03s)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 bash profiles/collect.sh r03r || exit 1
timeout -k 10 550 bash profiles/collect.sh r03s --workload silesia || exit 1
