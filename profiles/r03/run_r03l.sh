# round 3: run groups tolerate hash-collision members; parity + diag + zu trace
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_stream.py -m gpu -x -v --timeout 300 --timeout-method thread -k "golden or structured or silesia or long or every_level or finder or edge" > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 150 python tools/diag_big6.py zu 32 262144 > $OUT/d6_zu.txt 2>&1 || exit 1
timeout -k 10 150 python tools/diag_big6.py db 16 4194304 > $OUT/d6_db.txt 2>&1 || exit 1
A="--no-verify --no-decode --no-stream --no-shapes --cpu-seconds 0.2 --steps 3 --warmup 1"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/zu_trace -o t -- python3 $GRAFT_REPO_ROOT/bench.py $A --workload zeros_urandom > $GRAFT_REPO_ROOT/$OUT/zu_trace.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
