"""bench.pick_traffic: the roofline's `traffic` must come from a counter profile of the timed
kernel: a profile of this library build within 15 % of the live
kernel time (counter passes run at a lower clock), another build's only within 5 %, else
null with the reason."""
import json
import os

import bench


def _write(d, name, us, sha):
    os.makedirs(os.path.join(d, "profiles"), exist_ok=True)
    with open(os.path.join(d, "profiles", name), "w") as f:
        json.dump({"avg_kernel_us": us, "hbm_bytes_per_launch": us * 1000.0, "lib_sha1": sha}, f)


def test_same_build_preferred_within_its_tolerance(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "lib_sha1", lambda: "abc")
    _write(tmp_path, "r03_pmc_x.json", 445.0, "old")    # other build, within 5 %
    _write(tmp_path, "r04_pmc_x.json", 490.0, "abc")    # this build, 11 % slower (profiled)
    t, info = bench.pick_traffic("pmc_x.json", 441.5)
    assert info["file"].endswith("r04_pmc_x.json") and info["same_library"] and t == 490000.0


def test_other_build_needs_five_percent(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "lib_sha1", lambda: "abc")
    _write(tmp_path, "r03_pmc_x.json", 490.0, "old")
    t, info = bench.pick_traffic("pmc_x.json", 441.5)
    assert t is None and not info["accepted"] and "traffic null" in info["note"]
    _write(tmp_path, "r02_pmc_x.json", 450.0, "older")
    t, info = bench.pick_traffic("pmc_x.json", 441.5)
    assert t == 450000.0 and not info["same_library"]
