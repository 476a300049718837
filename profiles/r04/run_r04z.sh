# round 4: configs[4] kernel trace after the run jumps, and the shapes leg
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04z
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py --steps 5 --warmup 2 --no-stream --no-dict --cpu-seconds 0.2 > $OUT/shapes.json 2> $OUT/shapes.err || exit 1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/zu -o zu -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload zeros_urandom --steps 2 --warmup 1 --no-verify --no-decode --no-stream --no-dict --no-shapes --cpu-seconds 0.2 > $GRAFT_REPO_ROOT/$OUT/zu.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
