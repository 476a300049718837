"""CPU checks of the bench line's provenance: the roofline's `traffic` and issue rates come from the
newest committed PMC summary of the same workload (profiles/<tag>_pmc.json), tags ordered by round, then
r02a..r02z, r02aa..r02az, ... (a plain string sort would put r02o after r02bd, a length sort r03a before
r02bd)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (no GPU work at import)

DEFAULT_CFG = {"workload": "enwik8", "bytes_per_gpu": 100_000_000, "block_size": 65536, "level": 9}


def _tag_key(tag):
    return bench.pmc_tag_key(tag)


def test_tag_order():
    tags = ["r02o", "r02bd", "r03a", "r02av", "r03ab", "r03z", "r01h"]
    assert sorted(tags, key=_tag_key) == ["r01h", "r02o", "r02av", "r02bd", "r03a", "r03z", "r03ab"]


def test_pmc_traffic_takes_newest_tag_of_the_workload():
    got = bench.pmc_traffic(DEFAULT_CFG)
    assert got is not None
    path, rec = got
    tags = []
    for name in os.listdir(os.path.join(ROOT, "profiles")):
        if not name.endswith("_pmc.json"):
            continue
        with open(os.path.join(ROOT, "profiles", name)) as f:
            if json.load(f).get("config") == DEFAULT_CFG:
                tags.append(name[: -len("_pmc.json")])
    assert tags
    newest = max(tags, key=_tag_key)
    assert os.path.basename(path) == f"{newest}_pmc.json"
    # the record carries everything the roofline needs
    for k in ("avg_duration_us", "fetch_bytes_corrected", "write_bytes", "hbm_bytes_per_launch",
              "valu_per_simd_cycle", "salu_per_cu_cycle"):
        assert rec.get(k) is not None, k
    assert rec["hbm_bytes_per_launch"] == rec["fetch_bytes_corrected"] + rec["write_bytes"]


def test_pmc_traffic_none_for_unprofiled_workload():
    assert bench.pmc_traffic(dict(DEFAULT_CFG, level=3)) is None
