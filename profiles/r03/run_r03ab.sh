# round 3: k_find_sorted_hbm text from HBM/L2 (default now) + dictionary greedy/lazy walk in parallel:
# test_gpu.py whole, dictionary stream tests, dictionary timing
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03ab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_stream.py -m gpu -x -v --timeout 300 --timeout-method thread -k "dictionary" > $OUT/tests_dict.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/time_dict.py 8 > $OUT/dict.jsonl 2> $OUT/dict.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "not dictionary" > $OUT/tests_gpu.log 2>&1 || exit 1
echo done > $OUT/ok
