# round 4: dictionary shortcut rounds + legacy on the data-parallel path (tests), then the baseline bench and phase timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04b
mkdir -p $OUT
export TMPDIR=/tmp
python -c "import os;print(len(os.sched_getaffinity(0)), os.cpu_count())" > $OUT/cpus.txt; cat /sys/fs/cgroup/cpu.max >> $OUT/cpus.txt 2>&1; nproc >> $OUT/cpus.txt
timeout -k 10 600 python -u -m pytest tests/test_stream.py tests/test_gpu.py -m gpu -k "dict or legacy" -x -v --timeout 240 --timeout-method thread --durations=30 > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-shapes --no-stream --no-verify --cpu-seconds 1 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 python -u tools/diag_find.py 100 > $OUT/diag.txt 2>&1 || exit 1
echo done > $OUT/ok
