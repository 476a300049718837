#!/bin/bash
# Per-phase traffic of k_find_sorted on one shape: for each library variant (the product build and the
# SZ4_SKIP_* timing builds, tools/build_variant.sh), a kernel trace and separate PMC passes
# (FETCH_SIZE, WRITE_SIZE, TCC hit/miss) of tools/prof_shape.py.
#   bash profiles/phase_pmc.sh TAG SHAPE "variant ..."      (variant "base" = smallz4_amd/lib/libsmallz4_amd.so)
# Output: gpurun_out/TAG/<variant>_{trace,fetch,write,tcc}/ and .log files.  Each GPU step has its own
# time limit and the chain stops at the first failure.
set -euo pipefail
TAG=$1
SHAPE=$2
VARIANTS=${3:-base}
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 python3 "$R/tools/prof_shape.py" "$SHAPE" --reps 1 > "$OUT/gen.log" 2>&1
for v in $VARIANTS; do
  # a SZ4_SKIP_* build's pass-1 results are wrong: the pipeline stops after pass 1 (the later kernels would
  # read them), and so does the product build's run beside them ("base2")
  STOP=""
  if [ "$v" = base ]; then unset SMALLZ4_AMD_LIB
  elif [ "$v" = base2 ]; then unset SMALLZ4_AMD_LIB; STOP="--stop-after 2"
  else export SMALLZ4_AMD_LIB=$R/smallz4_amd/lib/libsmallz4_amd_$v.so; STOP="--stop-after 2"; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${v}_trace" -o run -- \
    python3 "$R/tools/prof_shape.py" "$SHAPE" --reps 3 $STOP > "$OUT/${v}_trace.log" 2>&1
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/${v}_fetch" -o run -- \
    python3 "$R/tools/prof_shape.py" "$SHAPE" --reps 1 $STOP > "$OUT/${v}_fetch.log" 2>&1
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/${v}_write" -o run -- \
    python3 "$R/tools/prof_shape.py" "$SHAPE" --reps 1 $STOP > "$OUT/${v}_write.log" 2>&1
  timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/${v}_tcc" -o run -- \
    python3 "$R/tools/prof_shape.py" "$SHAPE" --reps 1 $STOP > "$OUT/${v}_tcc.log" 2>&1
done
echo done > "$OUT/ok"
