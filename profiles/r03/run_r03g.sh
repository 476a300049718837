# round 3 final tree, part 2: profile collections (bench line with its shapes/stream/decode legs, kernel
# trace, FETCH/WRITE/SQ passes) for the headline workload (r03g) and the Silesia shape (r03h, configs[2])
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 bash profiles/collect.sh r03g || exit 1
timeout -k 10 550 bash profiles/collect.sh r03h --workload silesia || exit 1
