"""Times the greedy/lazy levels on inputs with long same-letter runs (the cases of
tests/test_gpu.py::test_greedy_lazy_long_runs and test_stream.py's carried-state chunks), one line of
JSON per case: seconds per call after a warm-up call.  GPU only; no oracle involved.

    python tools/time_runs.py [--lib path]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--only", default="", help="case,chain (e.g. runs_4m_stream,65535)")
    a = ap.parse_args()
    if a.lib:
        os.environ["SMALLZ4_AMD_LIB"] = a.lib
    import smallz4_amd
    from smallz4_amd import synth
    c = smallz4_amd.Compressor(device=0)
    M = 1 << 20
    runs4m = synth.enwik8_like((4 << 20) - 40000, seed=43) + bytes(140000) + synth.enwik8_like(10000, seed=44)
    carry = synth.enwik8_like(2 * 4 * M - 50000, seed=92) + bytes(120000) + synth.enwik8_like(4 * M, seed=93) + \
        bytes(90000) + synth.enwik8_like(2 * 4 * M + 12345, seed=94)
    cases = [("runs_b_1m_blocks", lambda ch: c.compress_blocks(bytes(70000) + synth.enwik8_like(5000, seed=42) + bytes(90000), 1 << 20, ch)),
             ("runs_4m_stream", lambda ch: c.lz4(runs4m, ch)),
             ("carry_20m_stream", lambda ch: c.lz4(carry, ch))]
    for name, fn in cases:
        for ch in (1, 3, 5, 9):
            chain = 65535 if ch == 9 else ch
            if a.only and a.only != f"{name},{chain}":
                continue
            fn(chain)
            t = time.time()
            fn(chain)
            print(json.dumps({"case": name, "level_chain": chain, "seconds": round(time.time() - t, 3)}), flush=True)


if __name__ == "__main__":
    main()
