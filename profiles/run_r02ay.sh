# round 2: parse regression on incompressible data -- kernel traces of random (100 MB, 64 KiB blocks) and zeros/urandom (256 MB, 256 KiB blocks), HEAD vs the tree before the parallel parse repair (66b9cc9)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02ay
mkdir -p $OUT
export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/smallz4_amd/lib
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 3 --warmup 1"
cd /tmp
for v in old new; do
  if [ $v = new ]; then lib=$L/libsmallz4_amd.so; else lib=$L/libsmallz4_amd_$v.so; fi
  for w in random zeros_urandom; do
    if [ $w = random ]; then X=""; else X="--mb 256"; fi
    SMALLZ4_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/${w}_$v -o bench -- \
      python3 $GRAFT_REPO_ROOT/bench.py $A --workload $w $X > $GRAFT_REPO_ROOT/$OUT/${w}_$v.json 2> $GRAFT_REPO_ROOT/$OUT/${w}_$v.err || exit 1
  done
done
echo done > $GRAFT_REPO_ROOT/$OUT/ok
