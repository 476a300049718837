# round 3: parallel parse repair for range-minimum blocks; parity + Silesia trace
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_stream.py -m gpu -x -v --timeout 300 --timeout-method thread -k "golden or structured or silesia or long or every_level or finder or edge or parse" > $OUT/tests.log 2>&1 || exit 1
A="--no-verify --no-decode --no-stream --no-shapes --cpu-seconds 0.2 --steps 3 --warmup 1"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/sil -o t -- python3 $GRAFT_REPO_ROOT/bench.py $A --workload silesia > $GRAFT_REPO_ROOT/$OUT/sil.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
