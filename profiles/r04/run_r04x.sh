# round 4: kernel traces of the slow long-run cases (4 MiB dependent blocks at -9, 20 MB at level 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04x
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/r9 -o r9 -- \
  python3 $GRAFT_REPO_ROOT/tools/time_runs.py --only runs_4m_stream,65535 > $GRAFT_REPO_ROOT/$OUT/r9.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/c1 -o c1 -- \
  python3 $GRAFT_REPO_ROOT/tools/time_runs.py --only carry_20m_stream,1 > $GRAFT_REPO_ROOT/$OUT/c1.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
