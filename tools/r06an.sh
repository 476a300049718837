#!/bin/bash
R=${GRAFT_REPO_ROOT:-$PWD}
O=gpurun_out/r06an
bash tools/gpu_steps.sh $O \
 "dtests|400|python -u -m pytest tests/test_stream.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k 'dict or Dict or dictionary'" \
 "dict|200|cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/dict -o run -- python3 $R/tools/time_dict.py 8"
 bash tools/gpu_steps.sh gpurun_out/r06an "smoke|200|python3 -c \"import __graft_entry__ as g; g.smoke()\""
