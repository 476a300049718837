# round 3: zeros/urandom kernel split; Silesia and enwik8-4m benches
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03v
mkdir -p $OUT
export TMPDIR=/tmp
A="--no-verify --no-decode --no-stream --no-shapes --cpu-seconds 0.2 --steps 3 --warmup 1"
timeout -k 10 300 python -u bench.py $A --workload silesia > $OUT/sil.json 2> $OUT/sil.err || exit 1
timeout -k 10 300 python -u bench.py $A --block-size 4194304 > $OUT/t4m.json 2> $OUT/t4m.err || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/zu -o t -- python3 $GRAFT_REPO_ROOT/bench.py $A --workload zeros_urandom --mb 268.435456 > $GRAFT_REPO_ROOT/$OUT/zu.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
