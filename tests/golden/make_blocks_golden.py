"""Regenerate tests/golden/blocks.json: independent-block fixtures from the REFERENCE itself.

The data-parallel entry point (sz4_compress_blocks_device) emits, per block, exactly what
smallz4::lz4 writes for that block alone.  For inputs whose blocks are too slow for the reference to
redo inside a GPU test (4 MiB blocks of binary records: ~2 minutes each at -9), this script runs the
reference (oracle/_ref/libsmallz4_ref.so, compiled in place from /root/reference) once, here, one
process per block, and records the SHA-256 of every block (size word + payload) and of the whole frame
(smallz4 header, blocks, end mark).  The inputs are generator specs (tests/golden/inputs.py) with their
SHA-256, so a generator change is caught.

    python tests/golden/make_blocks_golden.py [-j 8]
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

M = 4 << 20
HEADER = bytes([0x04, 0x22, 0x4D, 0x18, 0x40, 0x70, 0xDF])


def piece(kind, n, seed, index=0):
    return {"gen": "silesia_piece", "kind": kind, "n": n, "seed": seed, "index": index}


CASES = [
    # name, input spec, block size, maxChainLength
    ("db_4m", piece("db", 2 * M, 31), M, 65535),
    ("xml_4m", piece("xml", 2 * M, 32), M, 65535),
    ("exe_4m", piece("exe", 2 * M, 33), M, 65535),
    ("image_4m", piece("image", 2 * M, 34), M, 65535),
    ("src_4m", piece("src", 2 * M, 35), M, 65535),
    ("text_4m", {"gen": "enwik8_like", "n": 2 * M, "seed": 36}, M, 65535),
    ("silesia_mix_4m", {"gen": "silesia_like", "n": 3 * M, "seed": 37}, M, 65535),
    ("db_64k", piece("db", 1 << 20, 38), 65536, 65535),
    ("db_256k", piece("db", 1 << 20, 39), 262144, 65535),
    ("exe_64k", piece("exe", 1 << 20, 40), 65536, 65535),
    ("db_4m_l6", piece("db", M, 41), M, 6),
    ("zu_256k", {"gen": "zeros_urandom_range", "lo": 3 * (1 << 24) + 5 * (1 << 20) + 12345, "n": 8 << 20, "seed": 10},
     262144, 65535),
]
# the blocks tests/test_shards.py samples from configs[4]'s full-size slices (the reference needs ~13 s per
# zeros/urandom block: its chain walk is quadratic in a run), one case per block:
#   zu_slice_<i>: block i of rank 0's 1.25 GiB slice of the 10 GiB input;  zu_4g_<i>: block i of the
#   4 GiB one-call test (input from 3 GiB on)
ZU_BS = 262144
ZU_SLICE = [0, 1706, 3412, 5118, 5119]
ZU_4G = [1, 8195, 16383]
CASES += [(f"zu_slice_{i}", {"gen": "zeros_urandom_range", "lo": i * ZU_BS, "n": ZU_BS, "seed": 10}, ZU_BS, 65535)
          for i in ZU_SLICE]
CASES += [(f"zu_4g_{i}", {"gen": "zeros_urandom_range", "lo": (3 << 30) + i * ZU_BS, "n": ZU_BS, "seed": 10}, ZU_BS, 65535)
          for i in ZU_4G]


def _block(args):
    spec, off, bs, chain = args
    data = inputs.make(spec)[off:off + bs]
    t = time.time()
    out = pyoracle.ref_lz4(data, chain)[7:-4]  # this block's size word + payload
    return inputs.sha(out), len(out), time.time() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=os.cpu_count() or 4)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    if not pyoracle.ref_available():
        sys.exit("oracle/_ref/libsmallz4_ref.so missing: run `make -C oracle` with /root/reference present")
    path = os.path.join(HERE, "blocks.json")
    old = {}
    if os.path.exists(path):
        with open(path) as f:
            old = {c["name"]: c for c in json.load(f)["cases"]}
    jobs, meta = [], []
    for name, spec, bs, chain in CASES:
        if a.only and name not in a.only.split(","):
            continue
        data = inputs.make(spec)
        offs = list(range(0, len(data), bs))
        meta.append((name, spec, bs, chain, len(data), inputs.sha(data), len(jobs), len(offs)))
        jobs += [(spec, o, bs, chain) for o in offs]
    with ProcessPoolExecutor(max_workers=a.j) as ex:
        res = list(ex.map(_block, jobs))
    for name, spec, bs, chain, n, isha, j0, nb in meta:
        blocks = res[j0:j0 + nb]
        # frame = header + blocks + end mark: its hash from the block bytes would need them all; keep
        # the per-block hashes and lengths, and the frame length
        old[name] = {"name": name, "input": spec, "input_len": n, "input_sha256": isha, "block_size": bs,
                     "max_chain": chain, "block_sha256": [b[0] for b in blocks], "block_len": [b[1] for b in blocks],
                     "frame_len": 7 + sum(b[1] for b in blocks) + 4, "ref_seconds": round(sum(b[2] for b in blocks), 1)}
        print(f"{name:16s} {n:9d} B, {nb:3d} blocks of {bs}: {old[name]['frame_len']} B, "
              f"{old[name]['ref_seconds']} s of reference time", flush=True)
    with open(path, "w") as f:
        json.dump({"generator": "tests/golden/make_blocks_golden.py",
                   "reference": "gbonneau-hardent/smallz4 @ 2025-01-17, smallz4::lz4 per block via oracle/_ref",
                   "cases": [old[k] for k in sorted(old)]}, f, indent=1)


if __name__ == "__main__":
    main()
