# round 3: LPF groups + rest of the suite (shards, stream, decoder), the finder tests, kinds, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_stream.py tests/test_unlz4.py tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "not test_dictionary_mode and (golden_fixtures or structured or silesia or long or shapes or every_level or finder or shards or stream or unlz4 or batch or rank0 or chunk or dropin or decoder or dictionary)" > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u profiles/probe_shapes.py --mb 48 --block-size 4194304 --kinds text,xml,exe,db,image,src > $OUT/kinds_4m.jsonl 2> $OUT/kinds.err || exit 1
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
echo done > $OUT/ok
