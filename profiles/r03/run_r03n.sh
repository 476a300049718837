# round 3: Silesia-shaped configs[2] bench under a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03n
mkdir -p $OUT
export TMPDIR=/tmp
A="--no-verify --no-decode --no-stream --no-shapes --cpu-seconds 0.2 --steps 3 --warmup 1"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/sil -o t -- python3 $GRAFT_REPO_ROOT/bench.py $A --workload silesia > $GRAFT_REPO_ROOT/$OUT/sil.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
