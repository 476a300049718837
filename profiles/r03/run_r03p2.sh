# round 3: run-key detection of k_find_big's groups samples members across the group (the first and last
# can both be hash collisions): the slow configs[4] block, the 1.25 GiB slice by pieces, zero/run parity
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03p2
mkdir -p $OUT
export TMPDIR=/tmp
SMALLZ4_AMD_LIB=$GRAFT_REPO_ROOT/smallz4_amd/lib/libsmallz4_amd_diag.so timeout -k 10 200 python -u tools/zu_slow.py > $OUT/diag.jsonl 2> $OUT/diag.err || exit 1
timeout -k 10 300 python -u tools/zu_pieces.py 256 1280 > $OUT/pieces.jsonl 2> $OUT/pieces.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_shards.py -m gpu -x -v --timeout 300 --timeout-method thread -k "zero or run or structured or silesia or rank0 or golden" > $OUT/tests.log 2>&1 || exit 1
echo done > $OUT/ok
