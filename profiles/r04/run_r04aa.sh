# round 4: k_prep's serial replay wave-uniform from registers (no memory access on the position chain):
# timing on long runs, the compressor + stream parity tests, headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04aa
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/time_runs.py > $OUT/time_base.json 2> $OUT/time_base.err || exit 1
timeout -k 10 700 python3 -u -m pytest tests/test_gpu.py tests/test_stream.py -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --no-shapes --no-decode --cpu-seconds 0.2 > $OUT/head.json 2> $OUT/head.err || exit 1
echo done > $OUT/ok
