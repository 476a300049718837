# round 2: k_find_big (big key groups: left-maximal candidates + prefix maximum) -- new parity tests,
# per-kind probe, then the whole test_gpu suite and the bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02i
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -v --timeout 170 --timeout-method thread -k "structured or silesia" > $OUT/new_tests.log 2>&1 &&
timeout -k 10 200 python -u profiles/probe_shapes.py --mb 8 --block-size 4194304 > $OUT/kinds_4m.jsonl 2> $OUT/kinds_4m.err &&
timeout -k 10 200 python -u profiles/probe_shapes.py --mb 8 --block-size 65536 > $OUT/kinds_64k.jsonl 2> $OUT/kinds_64k.err &&
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-stream --cpu-seconds 1 > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 700 python -u -m pytest tests/test_gpu.py -x -v --timeout 170 --timeout-method thread -k "not structured and not silesia" > $OUT/gpu_tests.log 2>&1
