# round 4: profile collection on the current tree (bench line with every leg, kernel trace, PMC passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash profiles/collect.sh r04s
