# round 2: at two workgroups per CU -- filtered loops unrolled by two (xunroll) and no filter (xnofilt) vs default; SQ counters
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r02ap
mkdir -p $OUT
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 5 --warmup 2"
L=$GRAFT_REPO_ROOT/smallz4_amd/lib
for rep in 1 2; do
  for v in new xunroll xnofilt; do
    if [ $v = new ]; then lib=$L/libsmallz4_amd.so; else lib=$L/libsmallz4_amd_$v.so; fi
    SMALLZ4_AMD_LIB=$lib timeout -k 10 120 python -u bench.py $A > $OUT/ab_${v}_$rep.json 2> $OUT/ab_${v}_$rep.err || exit 1
  done
done
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
ARGS="--steps 3 --warmup 1 --no-verify --no-decode --no-stream --cpu-seconds 0.2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT \
  --kernel-include-regex k_find_sorted --output-format csv -d $OUT/sqA -o bench -- python3 $R/bench.py $ARGS > $OUT/sqA.log 2>&1
