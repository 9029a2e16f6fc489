"""bench.py reports roofline.traffic only from a PMC summary of the library build it loaded (a stale
round-4 summary was reported as the timed kernel's traffic).  CPU test of the selection rule."""
import json
import os

import bench


def _write(d, name, build, kernels=True):
    with open(os.path.join(d, "profiles", name), "w") as f:
        json.dump({"build_id": build, "kernels": {"HESS_M": {"traffic_bytes_per_launch": 1.0}} if kernels else {}}, f)


def test_traffic_only_from_matching_build(tmp_path, monkeypatch):
    os.makedirs(tmp_path / "profiles")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    t, note = bench.measured_traffic("abc")
    assert t is None and "none" in note
    _write(str(tmp_path), "r04_pmc_traffic.json", None)  # a summary without a build id (round 4's)
    _write(str(tmp_path), "r07_pmc_traffic.json", "other")
    t, note = bench.measured_traffic("abc")
    assert t is None and "r07_pmc_traffic.json" in note
    _write(str(tmp_path), "r05_pmc_traffic.json", "abc")
    t, note = bench.measured_traffic("abc")
    assert note is None and t["source"] == os.path.join("profiles", "r05_pmc_traffic.json") and t["build_id"] == "abc"


def test_committed_summary_matches_its_build():
    """The newest committed PMC summary names the build it profiled."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(bench.__file__), "profiles", "*_pmc_traffic.json")))
    with open(files[-1]) as f:
        t = json.load(f)
    assert len(t.get("build_id", "")) == 64 and t["kernels"]["HESS_M"]["traffic_bytes_per_launch"] > 0
