#!/bin/bash
# The drop-in stream path (smallz4::lz4 through include/smallz4_amd.hpp, 4 MiB dependent blocks in
# 64 MiB chunks) timed in C++: tools/bin/stream_threads (tests/cpp/stream_threads.cpp, built in-tree by
# hipcc) compresses <reps> x 100 MB of enwik8-shaped text at -9 and prints MB/s and the device
# footprint.  Usage (on the GPU box): bash tools/stream_big.sh OUTDIR [reps]
set -eo pipefail
OUT=$1
REPS=${2:-10}
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p "$OUT"
python3 -c "import sys; sys.path.insert(0, '$R'); from smallz4_amd import synth; open('/tmp/sz4_stream_base.bin', 'wb').write(synth.enwik8_like(100_000_000, seed=8))"
timeout -k 10 300 "$R/tools/bin/stream_threads" big 9 /tmp/sz4_stream_base.bin "$REPS" /dev/null > "$OUT/stream_big.json"
cat "$OUT/stream_big.json"
