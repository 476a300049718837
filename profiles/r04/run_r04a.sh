# round 4: baseline on this round's box -- bench (no shapes), separate-sort split with a kernel trace, per-wave phase timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04a
mkdir -p $OUT
export TMPDIR=/tmp
python -c "import os;print(len(os.sched_getaffinity(0)), os.cpu_count())" > $OUT/cpus.txt; cat /sys/fs/cgroup/cpu.max >> $OUT/cpus.txt 2>&1; nproc >> $OUT/cpus.txt
timeout -k 10 300 python -u bench.py --no-shapes --no-stream --no-verify --cpu-seconds 1 > $OUT/bench.json 2> $OUT/bench.err || exit 1
cd /tmp
SZ4_SEPARATE_SORT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/sep -o bench -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-verify --no-stream --no-shapes --no-decode --cpu-seconds 0.5 > $GRAFT_REPO_ROOT/$OUT/sep.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/diag_find.py 100 > $OUT/diag.txt 2>&1 || exit 1
echo done > $OUT/ok
