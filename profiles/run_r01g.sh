set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r01g_ab
A="--no-verify --no-decode --cpu-seconds 0.5 --steps 20"
for i in 1 2 3; do
  timeout -k 10 200 python bench.py $A > gpurun_out/r01g_ab/separate_$i.json 2>/dev/null || exit 1
  SZ4_FUSE_SORT=1 timeout -k 10 200 python bench.py $A > gpurun_out/r01g_ab/fused_$i.json 2>/dev/null || exit 1
done
bash profiles/collect.sh r01g
