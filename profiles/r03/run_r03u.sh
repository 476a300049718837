# round 3: one atomic per longBits word in k_find_big; parity + kinds + zu
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_stream.py -m gpu -x -v --timeout 300 --timeout-method thread -k "golden or structured or silesia or long or finder or edge" > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u profiles/probe_shapes.py --mb 32 --block-size 4194304 --kinds text,xml,exe,db,src,silesia > $OUT/kinds.jsonl 2> $OUT/kinds.err || exit 1
timeout -k 10 200 python -u profiles/probe_shapes.py --mb 64 --block-size 262144 --kinds zu >> $OUT/kinds.jsonl 2>> $OUT/kinds.err || exit 1
timeout -k 10 150 python tools/diag_big6.py zu 32 262144 > $OUT/d6_zu.txt 2>&1 || exit 1
echo done > $OUT/ok
