# round 4: dictionary shortcut rounds + legacy on the data-parallel path, the split decoder (tests), then
# the baseline bench (with the C++ stream leg and its decode) and the phase timeline of k_find_sorted
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04b
mkdir -p $OUT
export TMPDIR=/tmp
python -c "import os;print(len(os.sched_getaffinity(0)), os.cpu_count())" > $OUT/cpus.txt; cat /sys/fs/cgroup/cpu.max >> $OUT/cpus.txt 2>&1; nproc >> $OUT/cpus.txt
timeout -k 10 900 python -u -m pytest tests/test_stream.py tests/test_gpu.py tests/test_unlz4.py -m gpu -k "dict or legacy or unlz4" -v --timeout 300 --timeout-method thread --durations=40 > $OUT/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $OUT/tests.log
# a test failure is fine here (read the log); an abort, a fault or a time limit ends the call
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 400 python -u bench.py --no-shapes --no-verify --cpu-seconds 1 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 python -u tools/diag_find.py 100 > $OUT/diag.txt 2>&1 || exit 1
echo done > $OUT/ok
