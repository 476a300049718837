# round 4: everything pending in one call (GPU boxes are scarce): tests + bench (r04b), then the A/B runs
# r04e (k_find_sorted), r04f (dictionary run skip), r04c (configs[4] parse repair threshold)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash profiles/r04/run_r04b.sh && bash profiles/r04/run_r04e.sh && bash profiles/r04/run_r04f.sh && bash profiles/r04/run_r04c.sh
