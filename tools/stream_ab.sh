set -eo pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
python3 -c "import sys; sys.path.insert(0, '$R'); from smallz4_amd import synth; open('/tmp/sz4_stream_base.bin', 'wb').write(synth.enwik8_like(100_000_000, seed=8))"
for c in 67108864 268435456; do
  SZ4_STREAM_CHUNK=$c timeout -k 10 200 "$R/tools/bin/stream_threads" big 9 /tmp/sz4_stream_base.bin 10 /dev/null > "$R/gpurun_out/r05ad/stream_$c.json"
  tail -1 "$R/gpurun_out/r05ad/stream_$c.json"
done
