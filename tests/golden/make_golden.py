"""Regenerate tests/golden/golden.json from the REFERENCE itself.

Runs smallz4::lz4 compiled in place from /root/reference (oracle/_ref/
libsmallz4_ref.so, built by `make -C oracle`) on every fixture input and records
the output length and SHA-256 (full bytes for small frames).  Nothing from the
reference is copied: the fixtures are inputs (generator specs + input hashes)
and the reference's outputs.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import inputs  # noqa: E402

sys.path.insert(0, inputs.ROOT)
from oracle import pyoracle  # noqa: E402

M = 4 << 20
T9 = {"gen": "enwik8_like", "n": 9 << 20, "seed": 3}
ALL = [0, 1, 2, 3, 4, 5, 6, 7, 8, 65535]

CASES = [
    # name, input spec, levels, legacy variants, dictionary spec
    ("empty", {"gen": "hex", "hex": ""}, [0, 1, 65535], [0, 1], None),
    ("one", {"gen": "hex", "hex": "61"}, [0, 3, 65535], [0, 1], None),
    ("five", {"gen": "hex", "hex": "6162636465"}, [1, 65535], [0], None),
    ("eleven", {"gen": "repeat", "unit": "78", "count": 11}, [1, 65535], [0], None),
    ("twelve", {"gen": "hex", "hex": "616263646566616263646566"}, [1, 4, 65535], [0, 1], None),
    ("thirteen", {"gen": "hex", "hex": "61626361626361626361626361"}, [1, 4, 65535], [0], None),
    ("aaa30", {"gen": "repeat", "unit": "61", "count": 30}, ALL, [0], None),
    ("ab300", {"gen": "repeat", "unit": "616263642d", "count": 60}, ALL, [0, 1], None),
    ("text64k", {"gen": "enwik8_like", "n": 65536, "seed": 11}, ALL, [0, 1], None),
    ("text200k", {"gen": "enwik8_like", "n": 200000, "seed": 12}, [2, 6, 65535], [0], None),
    ("zeros64k", {"gen": "zeros", "n": 65536}, [7, 65535], [0], None),
    ("zeros70k", {"gen": "zeros", "n": 70000}, [8, 65535], [0], None),
    ("zu256k", {"gen": "zeros_urandom", "n": 262144, "run": 70000, "seed": 4}, [65535], [0], None),
    ("runs100k", {"gen": "runs", "n": 100000, "seed": 2}, [4, 65535], [0], None),
    ("alpha2", {"gen": "small_alphabet", "n": 100000, "k": 2, "seed": 5}, [3, 7, 65535], [0], None),
    ("alpha4", {"gen": "small_alphabet", "n": 100000, "k": 4, "seed": 6}, [65535], [0], None),
    ("random70k", {"gen": "random", "n": 70000, "seed": 7}, [1, 65535], [0, 1], None),
    ("text9m", T9, [6, 65535], [0, 1], None),
    ("text9m_cut", dict(T9, patch=[[M - 12, "20746865"]]), [65535], [0], None),
    ("tail5", {"gen": "enwik8_like", "n": M + 5, "seed": 3}, [65535], [0], None),
    ("tail13", {"gen": "enwik8_like", "n": M + 13, "seed": 3}, [2, 65535], [0], None),
    ("zeros_across_blocks", {"gen": "concat", "parts": [{"gen": "enwik8_like", "n": M - 40000, "seed": 9},
                                                        {"gen": "zeros", "n": 140000},
                                                        {"gen": "enwik8_like", "n": 300000, "seed": 10}]},
     [65535], [0], None),
    ("dict30k", {"gen": "enwik8_like", "n": 100000, "seed": 22}, [6, 65535], [0],
     {"gen": "enwik8_like", "n": 30000, "seed": 21}),
    ("dict64k", {"gen": "enwik8_like", "n": 100000, "seed": 23}, [65535], [0],
     {"gen": "enwik8_like", "n": 65536, "seed": 24}),
]


def main():
    if not pyoracle.ref_available():
        sys.exit("oracle/_ref/libsmallz4_ref.so missing: run `make -C oracle` with /root/reference present")
    out = []
    for name, spec, levels, legacies, dspec in CASES:
        data = inputs.make(spec)
        dic = inputs.make(dspec) if dspec else b""
        for level in levels:
            for legacy in legacies:
                t = time.time()
                frame = pyoracle.ref_lz4(data, level, dic, bool(legacy))
                rec = {"name": name, "input": spec, "input_len": len(data), "input_sha256": inputs.sha(data),
                       "level": level, "legacy": legacy, "out_len": len(frame), "out_sha256": inputs.sha(frame)}
                if dspec:
                    rec["dict"] = dspec
                    rec["dict_sha256"] = inputs.sha(dic)
                if len(frame) <= 600:
                    rec["out_hex"] = frame.hex()
                out.append(rec)
                print(f"{name:22s} level {level:5d} legacy {legacy}: {len(data):8d} -> {len(frame):8d}"
                      f"  ({time.time() - t:.1f}s)", flush=True)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py",
                   "reference": "gbonneau-hardent/smallz4 @ 2025-01-17, smallz4::lz4 via oracle/_ref",
                   "cases": out}, f, indent=1)
    print(len(out), "vectors")


if __name__ == "__main__":
    main()
