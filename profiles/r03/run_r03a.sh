# round 3 start: kernel traces of the non-headline shapes (Silesia 4 MiB, zeros/urandom 256 KiB, text 4 MiB)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03a
mkdir -p $OUT
export TMPDIR=/tmp
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 3 --warmup 1"
timeout -k 10 200 python -u bench.py $A --workload silesia > $OUT/silesia.json 2> $OUT/silesia.err || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/silesia_trace -o t -- python3 $GRAFT_REPO_ROOT/bench.py $A --workload silesia > $GRAFT_REPO_ROOT/$OUT/silesia_trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/zu_trace -o t -- python3 $GRAFT_REPO_ROOT/bench.py $A --workload zeros_urandom > $GRAFT_REPO_ROOT/$OUT/zu_trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/t4m_trace -o t -- python3 $GRAFT_REPO_ROOT/bench.py $A --block-size 4194304 --mb 64 > $GRAFT_REPO_ROOT/$OUT/t4m_trace.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
