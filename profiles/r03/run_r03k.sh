# round 3: run table in interval blocks, exact run lengths, LPF in blocks > 64 KiB; parity + perf + zu trace
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_stream.py tests/test_shards.py -m gpu -x -v --timeout 300 --timeout-method thread -k "golden or structured or silesia or long or shapes or every_level or finder or chunk or edge or rank0 or batch" > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u profiles/probe_shapes.py --mb 48 --block-size 4194304 --kinds text,xml,exe,db,image,src > $OUT/kinds_4m.jsonl 2> $OUT/kinds.err || exit 1
A="--no-verify --no-decode --no-stream --no-shapes --cpu-seconds 0.2 --steps 3 --warmup 1"
timeout -k 10 200 python -u bench.py $A > $OUT/enwik8.json 2> $OUT/enwik8.err || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/zu_trace -o t -- python3 $GRAFT_REPO_ROOT/bench.py $A --workload zeros_urandom > $GRAFT_REPO_ROOT/$OUT/zu_trace.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
