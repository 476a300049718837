# round 4: dictionary first-round guess (A/B), k_find_sorted filter variants (A/B), then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04h
mkdir -p $OUT
export TMPDIR=/tmp
A="--mb 1 --steps 1 --warmup 1 --no-stream --no-shapes --no-decode --no-verify --cpu-seconds 0.1"
timeout -k 10 300 python -u bench.py $A > $OUT/dict_guess.json 2> $OUT/dict_guess.err || exit 1
SZ4_DICT_NO_GUESS=1 timeout -k 10 300 python -u bench.py $A > $OUT/dict_noguess.json 2> $OUT/dict_noguess.err || exit 1
B="--steps 10 --warmup 3 --no-stream --no-dict --no-shapes --no-decode --no-verify --cpu-seconds 0.2"
for v in base fu1 f0; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 240 python -u bench.py $B > $OUT/find_$v.json 2> $OUT/find_$v.err || exit 1
done
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread --durations=60 > $OUT/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $OUT/tests.log
echo done > $OUT/ok
