# round 2: which Silesia-shaped content makes k_find_long9 slow (per-kind stage times)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02h
mkdir -p $OUT
timeout -k 10 300 python -u profiles/probe_shapes.py --mb 8 --block-size 4194304 > $OUT/kinds_4m.jsonl 2> $OUT/kinds_4m.err &&
timeout -k 10 300 python -u profiles/probe_shapes.py --mb 8 --block-size 65536 > $OUT/kinds_64k.jsonl 2> $OUT/kinds_64k.err
