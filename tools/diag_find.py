#!/usr/bin/env python3
"""Diagnostic (python3 tools/diag_find.py MB [max_chain] [enwik8|zu|silesia]): k_find_sorted's per-wavefront counters from a SZ4_DIAG=3 build of the library
(smallz4_amd/lib/libsmallz4_amd_diag3.so, built by tools/build_diag.sh 3): below-chunk candidate steps
(dB), shift-register steps (dL), improve calls (dBi), extension steps (dLi) and cycles per wave."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["SMALLZ4_AMD_LIB"] = os.path.join(ROOT, "smallz4_amd", "lib", "libsmallz4_amd_diag3.so")
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import smallz4_amd  # noqa: E402
from smallz4_amd import synth  # noqa: E402

mb = float(sys.argv[1]) if len(sys.argv) > 1 else 100
chain = int(sys.argv[2]) if len(sys.argv) > 2 else 65535
workload = sys.argv[3] if len(sys.argv) > 3 else "enwik8"
n = int(mb * 1e6)
if workload == "zu":  # configs[4]: zeros/urandom at 256 KiB blocks
    data, bs = synth.zeros_urandom_range(0, n, seed=10), 262144
elif workload == "silesia":  # configs[2] at 4 MiB blocks
    data, bs = synth.silesia_like(n, seed=2), 4 << 20
else:
    data, bs = synth.enwik8_like(n, seed=8), 65536
comp = smallz4_amd.Compressor()
comp.compress_blocks(data[:1 << 22], bs, chain)
comp.set_timing(True)
comp.compress_blocks(data, bs, chain)
find_ms = comp.last_stage_ms()['find_sorted']
lib = comp._lib
lib.sz4_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
nwaves = min((n + 65535) // 65536, 1 << 17) * 16  # 16 waves per 64 Ki-target segment
buf = np.zeros(nwaves * 8, dtype=np.uint64)
assert lib.sz4_diag_read(buf.ctypes.data, buf.size) == 0
d = buf.reshape(-1, 8).astype(np.float64)
cyc = d[:, 1] - d[:, 0]
print(f"waves {nwaves}: below-chunk steps dB {d[:, 2].sum():.4g}, shift steps dL {d[:, 3].sum():.4g}, "
      f"broadcast steps serving <= 32 lanes {d[:, 4].sum():.4g}, <= 8 lanes {d[:, 5].sum():.4g}")
print(f"per wave: dB {d[:, 2].mean():.1f} dL {d[:, 3].mean():.1f}; cycles mean {cyc.mean():.4g} max {cyc.max():.4g}")
t_entry, t_search = d[:, 6], d[:, 7]
ok = t_entry > 0
span = d[ok, 1].max() - t_entry[ok].min()
print(f"phases per wave (ticks): sort {(d[ok, 0] - t_entry[ok]).mean():.4g}, "
      f"window load + search {(t_search[ok] - d[ok, 0]).mean():.4g}, text-order output {(d[ok, 1] - t_search[ok]).mean():.4g}; "
      f"kernel span {span:.4g} ticks in {find_ms:.3f} ms -> {span / find_ms / 1e6:.3f} GHz")
print(f"per position: dB {d[:, 2].sum() / n:.3f} dL {d[:, 3].sum() / n:.3f} (wave-steps per target position)")
print(f"hit branches per position {d[:, 4].sum() / n:.3f}; broadcast blocks {(buf.reshape(-1, 8)[:, 5] >> np.uint64(46)).sum() / n:.4f}/pos, flush rounds {((buf.reshape(-1, 8)[:, 5] >> np.uint64(30)) & np.uint64(0xFFFF)).sum() / n:.4f}/pos, extension lane-steps {(buf.reshape(-1, 8)[:, 5] & np.uint64(0x3FFFFFFF)).sum() / n:.3f}/pos")
