# round 3: LPF threshold A/B (text at 4 MiB blocks regressed 4867 -> 3566 MB/s once LPF targets >= 256
# went to k_find_big); data-parallel dictionary mode: parity + throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03y
mkdir -p $OUT
export TMPDIR=/tmp
for v in base lpf1k lpf4k lpf8k; do
  if [ $v = base ]; then L=smallz4_amd/lib/libsmallz4_amd.so; else L=smallz4_amd/lib/libsmallz4_amd_$v.so; fi
  SMALLZ4_AMD_LIB=$L timeout -k 10 200 python -u profiles/probe_shapes.py --mb 32 --block-size 4194304 --kinds text,xml,exe,db,src,silesia > $OUT/$v.jsonl 2> $OUT/$v.err || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_stream.py -m gpu -x -v --timeout 300 --timeout-method thread -k "dictionary or golden" > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/time_dict.py 8 > $OUT/dict.jsonl 2> $OUT/dict.err || exit 1
echo done > $OUT/ok
