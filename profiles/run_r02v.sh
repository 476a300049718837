# round 2: k_find_big resolve launch -- structured/Silesia parity, per-kind probe + trace on binary records, Silesia bench
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -x -v --timeout 170 --timeout-method thread -k "structured or silesia or long_matches or other_block_sizes or shapes" > $OUT/tests.log 2>&1 &&
timeout -k 10 200 python -u profiles/probe_shapes.py --mb 8 --block-size 4194304 --kinds db,xml,text > $OUT/kinds_4m.jsonl 2> $OUT/kinds_4m.err &&
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_db -o t -- python3 $GRAFT_REPO_ROOT/profiles/probe_shapes.py --mb 8 --block-size 4194304 --kinds db > $GRAFT_REPO_ROOT/$OUT/trace_db.log 2>&1) &&
timeout -k 10 300 python -u bench.py --workload silesia --no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 3 --warmup 1 > $OUT/silesia.json 2> $OUT/silesia.err
