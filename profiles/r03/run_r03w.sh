# round 3: parallel rmq repair only in long blocks; 256 MiB batch pieces; parity + zu/silesia benches
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03w
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "golden or structured or silesia or long or zero" > $OUT/tests.log 2>&1 || exit 1
A="--no-verify --no-decode --no-stream --no-shapes --cpu-seconds 0.2 --steps 3 --warmup 1"
timeout -k 10 300 python -u bench.py $A --workload zeros_urandom --mb 268.435456 > $OUT/zu.json 2> $OUT/zu.err || exit 1
timeout -k 10 300 python -u bench.py $A --workload silesia > $OUT/sil.json 2> $OUT/sil.err || exit 1
echo done > $OUT/ok
