# round 2: lazy replay with mbcnt selection -- greedy/lazy parity, level-6 bench, dictionary-mode timing
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02u
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 170 --timeout-method thread -k "every_level or greedy_lazy or golden or stream_multiblock or edge or shapes" > $OUT/lazy_tests.log 2>&1 &&
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 5 --warmup 2"
timeout -k 10 200 python -u bench.py $A --level 6 > $OUT/enwik8_l6.json 2> $OUT/enwik8_l6.err &&
timeout -k 10 200 python -u bench.py $A --level 5 > $OUT/enwik8_l5.json 2> $OUT/enwik8_l5.err &&
timeout -k 10 300 python -u tools/time_dict.py 8 > $OUT/dict.jsonl 2> $OUT/dict.err
