"""Regenerate tests/golden/streams.json: whole-stream fixtures (smallz4::lz4 over the input, with its
dictionary and frame format) from the REFERENCE itself.

Some stream cases cost the reference too long to redo inside a GPU test: a long run of one byte value
makes its chain walk quadratic (every position after the same-letter shortcut walks up to 65535
candidates, smallz4.h:173-255), and configs[4]-shaped data has hundreds of such runs.  This script
runs the reference (oracle/_ref/libsmallz4_ref.so, compiled in place from /root/reference) once, here,
one process per case, and records the SHA-256 and length of each frame.  Inputs and dictionaries are
generator specs (tests/golden/inputs.py) with their SHA-256, so a generator change is caught.

    python tests/golden/make_streams_golden.py [-j 8] [--only name,...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import inputs  # noqa: E402

sys.path.insert(0, inputs.ROOT)
from oracle import pyoracle  # noqa: E402

M = 1 << 20


def text(n, seed):
    return {"gen": "enwik8_like", "n": n, "seed": seed}


def zeros(n):
    return {"gen": "zeros", "n": n}


def cat(*parts):
    return {"gen": "concat", "parts": list(parts)}


# a run of 65400 equal bytes whose staged start (after the 65535-byte dictionary prefix) is 100 bytes
# past a 32 KiB boundary: it holds no aligned 32 KiB window, yet it is long enough for the shortcut
UNLUCKY = cat(text(32768 * 5 + 101, 75), {"gen": "repeat", "unit": "00", "count": 65400}, text(300000, 76))
ZERO_RUN_8M = cat(text(3_900_000, 80), zeros(200_000), text(3_900_000, 81))

def hexs(b):
    return {"gen": "hex", "hex": b.hex()}


def skip_into_run(seed):
    """tests/test_gpu.py's _skip_into_run: a long match that ends 10 bytes into a 100 KB zero run."""
    import numpy as np
    r = np.random.default_rng(seed).integers(1, 256, size=1000, dtype=np.uint8).tobytes()
    return cat(text(3000, seed), hexs(r), zeros(10), hexs(b"xyz"), hexs(r), zeros(100000), text(20000, seed + 1))


RUNS_A = cat(text(30000, 41), zeros(150000))
RUNS_B = cat(zeros(70000), text(5000, 42), zeros(90000))
RUNS_4M = cat(text((4 << 20) - 40000, 43), zeros(140000), text(10000, 44))
SHORTCUT_256K = cat(text(30000, 9), zeros(150000), text(82144, 10))
CARRY = cat(text(2 * 4 * M - 50000, 92), zeros(120000), text(4 * M, 93), zeros(90000), text(2 * 4 * M + 12345, 94))

# independent-block frames (the smallz4 header, every block as smallz4::lz4 writes it alone, the end
# mark): name, input spec, block size, maxChainLength -- the cases of test_gpu.py that run the oracle on
# zero runs (quadratic for the reference: its chain walk visits the whole run)
BLOCK_CASES = []
for _ch in range(1, 7):
    BLOCK_CASES += [(f"gl_skip_into_run_l{_ch}", skip_into_run(40), 262144, _ch),
                    (f"gl_runs_a_l{_ch}", RUNS_A, 262144, _ch),
                    (f"gl_runs_b_l{_ch}", RUNS_B, 1 << 20, _ch)]
for _ch in (7, 8, 65535):
    BLOCK_CASES.append((f"shortcut_256k_l{_ch}", SHORTCUT_256K, 262144, _ch))

CASES = [
    # name, input spec, dictionary spec (or None), maxChainLength, legacy
    ("dict_zero_run_8m_l9", ZERO_RUN_8M, text(65536, 82), 65535, False),
    ("dict_zero_run_8m_l6", ZERO_RUN_8M, text(65536, 82), 6, False),
    ("dict_unlucky_run_l9", UNLUCKY, text(20000, 77), 65535, False),
    ("dict_unlucky_run_l6", UNLUCKY, text(20000, 77), 6, False),
    ("dict_unlucky_run_l3", UNLUCKY, text(20000, 77), 3, False),
    ("dict_runs_multi_block_l9", cat(text(4 * M - 70000, 83), zeros(150000), text(M, 84),
                                     {"gen": "repeat", "unit": "61", "count": 70000}, text(2 * M, 85)),
     text(40000, 86), 65535, False),
    ("dict_legacy_12m_l9", cat(text(7 * M, 87), zeros(100000), text(5 * M, 88)), text(65536, 89), 65535, True),
    ("dict_legacy_12m_l3", cat(text(7 * M, 87), zeros(100000), text(5 * M, 88)), text(65536, 89), 3, True),
    ("dict_zeros_urandom_l9", {"gen": "zeros_urandom_range", "lo": 5 << 20, "n": 6 * M, "seed": 10}, text(65536, 90),
     65535, False),
] + [(f"gl_runs_4m_l{_ch}", RUNS_4M, None, _ch, False) for _ch in range(1, 7)] + \
    [(f"carry_state_l{_ch}", CARRY, None, _ch, False) for _ch in (1, 3, 5, 65535)]


def _block_case(args):
    name, spec, bs, chain = args
    data = inputs.make(spec)
    t = time.time()
    frame = bytes([0x04, 0x22, 0x4D, 0x18, 0x40, 0x70, 0xDF])
    for o in range(0, len(data), bs):
        frame += pyoracle.ref_lz4(data[o:o + bs], chain)[7:-4]
    frame += bytes(4)
    return {"name": name, "kind": "blocks", "input": spec, "input_len": len(data), "input_sha256": inputs.sha(data),
            "block_size": bs, "dictionary": None, "dictionary_sha256": inputs.sha(b""), "max_chain": chain, "legacy": False,
            "frame_len": len(frame), "frame_sha256": inputs.sha(frame), "ref_seconds": round(time.time() - t, 1)}


def _case(args):
    if len(args) == 4:
        return _block_case(args)
    name, spec, dspec, chain, legacy = args
    data = inputs.make(spec)
    dic = inputs.make(dspec) if dspec else b""
    t = time.time()
    out = pyoracle.ref_lz4(data, chain, dic, legacy)
    return {"name": name, "kind": "stream", "input": spec, "input_len": len(data), "input_sha256": inputs.sha(data),
            "dictionary": dspec, "dictionary_sha256": inputs.sha(dic), "max_chain": chain, "legacy": legacy,
            "frame_len": len(out), "frame_sha256": inputs.sha(out), "ref_seconds": round(time.time() - t, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=os.cpu_count() or 4)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    if not pyoracle.ref_available():
        sys.exit("oracle/_ref/libsmallz4_ref.so missing: run `make -C oracle` with /root/reference present")
    path = os.path.join(HERE, "streams.json")
    old = {}
    if os.path.exists(path):
        with open(path) as f:
            old = {c["name"]: c for c in json.load(f)["cases"]}
    jobs = [c for c in CASES + BLOCK_CASES if not a.only or c[0] in a.only.split(",")]
    with ProcessPoolExecutor(max_workers=a.j) as ex:
        for rec in ex.map(_case, jobs):
            old[rec["name"]] = rec
            print(f"{rec['name']:28s} {rec['input_len']:9d} B -> {rec['frame_len']:9d} B, "
                  f"{rec['ref_seconds']} s of reference time", flush=True)
    with open(path, "w") as f:
        json.dump({"generator": "tests/golden/make_streams_golden.py",
                   "reference": "gbonneau-hardent/smallz4 @ 2025-01-17, smallz4::lz4 (stream, dictionary, legacy) "
                                "via oracle/_ref",
                   "cases": [old[k] for k in sorted(old)]}, f, indent=1)


if __name__ == "__main__":
    main()
