# round 3: run table v2 (run index via lm, cooperative walk) -- parity on the block fixtures and structured content, then the shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 170 --timeout-method thread -k "golden_fixtures or structured or silesia or long_matches or shapes or every_level or finder or long_run" > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u profiles/probe_shapes.py --mb 48 --block-size 4194304 --kinds text,xml,exe,db,image,src > $OUT/kinds_4m.jsonl 2> $OUT/kinds.err || exit 1
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 3 --warmup 1"
timeout -k 10 200 python -u bench.py $A --workload silesia > $OUT/silesia.json 2> $OUT/silesia.err || exit 1
echo done > $OUT/ok
