# round 2: k_find_sorted split into k_find_sorted_lds (SGPR budget 80: two workgroups per CU) and _hbm (96) -- bench, parity
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02ao
mkdir -p $OUT
A="--no-verify --no-decode --no-stream --cpu-seconds 0.2 --steps 5 --warmup 2"
timeout -k 10 120 python -u bench.py $A > $OUT/ab_new.json 2> $OUT/ab_new.err || exit 1
timeout -k 10 120 python -u bench.py $A --block-size 4194304 --mb 64 > $OUT/ab4m_new.json 2> $OUT/ab4m_new.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_stream.py -x -v --timeout 170 --timeout-method thread -k "every_level or shapes or edge_sizes or other_block_sizes or silesia or structured or stream_multiblock or golden or run_across or chunk_boundaries or long_matches or finder_intermediate or dictionary or greedy or headers" > $OUT/tests.log 2>&1
