bash tools/gpu_steps.sh gpurun_out/r06c \
 "tests|400|python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_unlz4.py tests/test_memory.py" \
 "phase|700|bash profiles/phase_pmc.sh r06c silesia 'base old skipsearch skipbcast skipshift'" \
 "diag|150|python3 tools/diag_find.py 211.93858 65535 silesia"
