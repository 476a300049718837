# round 3: kernel split of configs[4] (268 MB of the slice) and text at 4 MiB blocks on the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03t2
mkdir -p $OUT
export TMPDIR=/tmp
A="--no-verify --no-decode --no-stream --no-shapes --cpu-seconds 0.2 --steps 3 --warmup 1"
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/zu -o t -- python3 $GRAFT_REPO_ROOT/bench.py $A --workload zeros_urandom --mb 268.435456 > $GRAFT_REPO_ROOT/$OUT/zu.json 2> $GRAFT_REPO_ROOT/$OUT/zu.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/t4m -o t -- python3 $GRAFT_REPO_ROOT/bench.py $A --block-size 4194304 > $GRAFT_REPO_ROOT/$OUT/t4m.json 2> $GRAFT_REPO_ROOT/$OUT/t4m.err || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
