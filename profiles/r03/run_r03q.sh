# round 3: where find_long goes on text at 4 MiB blocks
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 150 python tools/diag_big6.py text 32 4194304 > $OUT/d6_text.txt 2>&1 || exit 1
timeout -k 10 150 python tools/diag_big6.py xml 16 4194304 > $OUT/d6_xml.txt 2>&1 || exit 1
A="--no-verify --no-decode --no-stream --no-shapes --cpu-seconds 0.2 --steps 3 --warmup 1"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/t4m -o t -- python3 $GRAFT_REPO_ROOT/bench.py $A --block-size 4194304 > $GRAFT_REPO_ROOT/$OUT/t4m.log 2>&1 || exit 1
echo done > $GRAFT_REPO_ROOT/$OUT/ok
