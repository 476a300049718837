# round 3: capped run-key targets handed to k_find_big; parity + diag + zu/silesia/text benches
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 150 python tools/diag_long9.py 64 > $OUT/d5zu.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "golden or structured or silesia or long or zero" > $OUT/tests.log 2>&1 || exit 1
A="--no-verify --no-decode --no-stream --no-shapes --cpu-seconds 0.2 --steps 3 --warmup 1"
timeout -k 10 300 python -u bench.py $A --workload zeros_urandom --mb 268.435456 > $OUT/zu.json 2> $OUT/zu.err || exit 1
timeout -k 10 300 python -u bench.py $A --workload silesia > $OUT/sil.json 2> $OUT/sil.err || exit 1
timeout -k 10 300 python -u bench.py $A --block-size 4194304 > $OUT/t4m.json 2> $OUT/t4m.err || exit 1
echo done > $OUT/ok
