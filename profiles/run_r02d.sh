# round 2: kernel profile of the default workload (trace + PMC passes), the lazy levels' trace,
# and the other BASELINE shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02d_shapes
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 170 --timeout-method thread -k "every_level or greedy_lazy or golden or stream_multiblock" > $OUT/lazy_tests.log 2>&1 &&
bash profiles/collect.sh r02d &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_l6 -o l6 -- python3 $GRAFT_REPO_ROOT/bench.py --level 6 --steps 5 --warmup 2 --no-verify --no-decode --no-stream --cpu-seconds 0.5 > $GRAFT_REPO_ROOT/$OUT/trace_l6.log 2>&1) &&
A="--no-verify --no-decode --no-stream --cpu-seconds 0.5 --steps 3 --warmup 1"
for w in random zeros_urandom silesia; do
  timeout -k 10 300 python -u bench.py $A --workload $w > $OUT/$w.json 2> $OUT/$w.err || exit 1
done
timeout -k 10 200 python -u bench.py $A --workload enwik8 --block-size 4194304 --mb 64 > $OUT/enwik8_4m.json 2>/dev/null
