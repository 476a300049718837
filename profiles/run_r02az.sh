# round 2: k_dp_fix<false> restore without __threadfence (workgroup fence) -- test_gpu.py, random / zeros-urandom / headline benches, random kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02az
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 170 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 3 --warmup 1"
timeout -k 10 200 python -u bench.py $A --workload random > $OUT/random.json 2> $OUT/random.err || exit 1
timeout -k 10 300 python -u bench.py $A --workload zeros_urandom > $OUT/zeros_urandom.json 2> $OUT/zeros_urandom.err || exit 1
timeout -k 10 200 python -u bench.py --no-stream --cpu-seconds 0.2 --steps 5 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/random_trace -o bench -- \
  python3 $GRAFT_REPO_ROOT/bench.py $A --workload random > $GRAFT_REPO_ROOT/$OUT/random_trace.log 2>&1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
