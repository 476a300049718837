# round 4: the broadcast specialisation in the LDS-window kernel only (k_find_sorted_hbm keeps 64 VGPRs):
# compressor parity tests, bench with shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04ad
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/test_gpu.log 2>&1 || exit 1
timeout -k 10 600 python3 -u bench.py --steps 10 --warmup 3 --no-stream --no-dict --cpu-seconds 0.2 > $OUT/shapes.json 2> $OUT/shapes.err || exit 1
echo done > $OUT/ok
