set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r01h_shapes
A="--no-verify --no-decode --cpu-seconds 0.5 --steps 3 --warmup 1"
timeout -k 10 200 python bench.py $A --mb 64 --block-size 4194304 > gpurun_out/r01h_shapes/enwik8_4m.json 2>/dev/null && \
timeout -k 10 200 python bench.py $A --data zeros_urandom --block-size 262144 > gpurun_out/r01h_shapes/zeros_urandom_256k.json 2>/dev/null && \
timeout -k 10 200 python bench.py $A --data zeros > gpurun_out/r01h_shapes/zeros_64k.json 2>/dev/null && \
timeout -k 10 200 python bench.py $A --data random > gpurun_out/r01h_shapes/random_64k.json 2>/dev/null && \
timeout -k 10 200 python bench.py --no-verify --cpu-seconds 0.5 --steps 3 --warmup 1 --level 6 > gpurun_out/r01h_shapes/enwik8_l6.json 2>/dev/null
