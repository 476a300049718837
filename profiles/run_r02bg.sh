# round 2: final tree -- the driver's default bench line and the 4 MiB shape
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02bg
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 120 python -u bench.py --no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 10 --warmup 3 --block-size 4194304 --mb 64 > $OUT/enwik8_4m.json 2> $OUT/enwik8_4m.err || exit 1
echo done > $OUT/ok
