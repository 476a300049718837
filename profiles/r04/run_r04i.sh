# round 4: the fixture-based slow tests and the decoder index change, split decode A/B on 64 KiB blocks,
# the full default bench (all legs), then the profile collection of the headline workload
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_stream.py tests/test_unlz4.py -m gpu -k "greedy_lazy or long_run_shortcut or carry_state or unlz4" -v --timeout 300 --timeout-method thread --durations=20 > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $OUT/tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
B="--steps 10 --warmup 3 --no-stream --no-dict --no-shapes --no-verify --cpu-seconds 0.2"
SZ4_UNLZ4_SPLIT=1 timeout -k 10 240 python -u bench.py $B > $OUT/split1.json 2> $OUT/split1.err || exit 1
timeout -k 10 240 python -u bench.py $B > $OUT/split_auto.json 2> $OUT/split_auto.err || exit 1
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 900 bash profiles/collect.sh r04i_prof || exit 1
echo done > $OUT/ok
