"""Deterministic fixture inputs: a spec (generator name + arguments) -> bytes.

Shared by make_golden.py (which runs the reference on them) and the tests.  The
SHA-256 of every generated input is stored in golden.json, so a change to a
generator is caught instead of silently shifting the expected outputs."""
from __future__ import annotations

import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from smallz4_amd import synth  # noqa: E402


def make(spec: dict) -> bytes:
    kind = spec["gen"]
    if kind == "hex":
        data = bytes.fromhex(spec["hex"])
    elif kind == "repeat":
        data = bytes.fromhex(spec["unit"]) * spec["count"]
    elif kind == "enwik8_like":
        data = synth.enwik8_like(spec["n"], seed=spec["seed"])
    elif kind == "zeros":
        data = bytes(spec["n"])
    elif kind == "zeros_urandom":
        data = synth.zeros_urandom(spec["n"], run=spec["run"], seed=spec["seed"])
    elif kind == "random":
        data = synth.random_bytes(spec["n"], seed=spec["seed"])
    elif kind == "small_alphabet":
        data = synth.small_alphabet(spec["n"], k=spec["k"], seed=spec["seed"])
    elif kind == "runs":
        data = synth.runs(spec["n"], seed=spec["seed"], max_run=spec.get("max_run", 3000))
    elif kind == "silesia_piece":
        data = synth._silesia_piece((spec["kind"], spec["n"], spec["seed"], spec.get("index", 0)))
    elif kind == "silesia_like":
        data = synth.silesia_like(spec["n"], seed=spec["seed"], workers=spec.get("workers", 1))
    elif kind == "zeros_urandom_range":
        data = synth.zeros_urandom_range(spec["lo"], spec["lo"] + spec["n"], seed=spec["seed"])
    elif kind == "concat":
        data = b"".join(make(p) for p in spec["parts"])
    else:
        raise ValueError(kind)
    if "patch" in spec:
        buf = bytearray(data)
        for off, hx in spec["patch"]:
            b = bytes.fromhex(hx)
            buf[off:off + len(b)] = b
        data = bytes(buf)
    return data


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()
