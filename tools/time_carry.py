#!/usr/bin/env python3
"""Times smallz4::lz4 on the carry_state fixtures (21 MB with long zero runs; tests/test_gpu.py's
test_greedy_lazy_long_runs) at -1/-3/-5, best of 3, and checks the frames against the fixture."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import inputs  # noqa: E402

import smallz4_amd  # noqa: E402


def main():
    with open(os.path.join(ROOT, "tests", "golden", "streams.json")) as f:
        cases = {c["name"]: c for c in json.load(f)["cases"]}
    comp = smallz4_amd.Compressor()
    for chain in (1, 3, 5):
        case = cases[f"carry_state_l{chain}"]
        data = inputs.make(case["input"])
        comp.lz4(data[:1 << 20], chain)
        best = 1e9
        for _ in range(3):
            t = time.perf_counter()
            out = comp.lz4(data, chain)
            best = min(best, time.perf_counter() - t)
        ok = len(out) == case["frame_len"] and inputs.sha(out) == case["frame_sha256"]
        print(f"carry_state_l{chain}: {len(data) / 1e6:.1f} MB best {best:.3f} s, frame equal {ok}", flush=True)


if __name__ == "__main__":
    main()
