# round 2: where k_find_sorted's time goes (separate sort launch), and kernel traces of the 4 MiB and level-6 shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02n
mkdir -p $OUT
export TMPDIR=/tmp
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 5 --warmup 2"
SZ4_SEPARATE_SORT=1 timeout -k 10 200 python -u bench.py $A > $OUT/separate_sort.json 2> $OUT/separate_sort.err &&
timeout -k 10 200 python -u bench.py $A > $OUT/fused.json 2> $OUT/fused.err &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_4m -o t -- python3 $GRAFT_REPO_ROOT/bench.py $A --block-size 4194304 --mb 64 > $GRAFT_REPO_ROOT/$OUT/trace_4m.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_l6 -o t -- python3 $GRAFT_REPO_ROOT/bench.py $A --level 6 > $GRAFT_REPO_ROOT/$OUT/trace_l6.log 2>&1
