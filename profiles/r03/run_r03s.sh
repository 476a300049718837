# round 3: ordered run buckets (nearest-first same-R search); parity + kinds + diag
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03s
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_stream.py -m gpu -x -v --timeout 300 --timeout-method thread -k "golden or structured or silesia or long or every_level or finder or edge" > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u profiles/probe_shapes.py --mb 32 --block-size 4194304 --kinds text,xml,exe,db,src,silesia > $OUT/kinds.jsonl 2> $OUT/kinds.err || exit 1
timeout -k 10 150 python tools/diag_big6.py text 32 4194304 > $OUT/d6_text.txt 2>&1 || exit 1
echo done > $OUT/ok
