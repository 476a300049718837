# round 2: k_find_sorted diagnostic counters, then the profile of HEAD (trace + PMC passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02o
mkdir -p $OUT
timeout -k 10 200 python -u tools/diag_find.py 100 > $OUT/diag.txt 2>&1 &&
bash profiles/collect.sh r02o
