# round 4: r04i then r04j in one call
set -o pipefail
cd $GRAFT_REPO_ROOT
bash profiles/r04/run_r04i.sh && bash profiles/r04/run_r04j.sh
