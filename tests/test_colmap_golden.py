"""COLMAP converter parity against the reference script's own outputs.

tests/golden/colmap_*.json hold seeded synthetic sparse models (text and binary encodings, pinhole and
SPHERE, max_d = 0 and fixed, several top_k / min_shared / theta0 / interval_scale settings) together
with the cams/*_cam.txt and pair.txt that colmap2mvsnet_acm.py's process_scene (:249-406) wrote for
them (scripts/make_colmap_golden.py, run where /root/reference exists).  acmmp.colmap must write the
same bytes: depth ranges (:183-217), k-d tree candidates, greedy shared-track bins, the angle filter
and the neighbour order of np.argsort (:302-363), the str() formatting of every float (:366-397)."""
import base64
import glob
import json
import os

import pytest

from acmmp import colmap

FIXTURES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "colmap_*.json")))


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p)[7:-5] for p in FIXTURES])
def test_converter_matches_reference_outputs(tmp_path, path):
    fx = json.load(open(path))
    src = tmp_path / "colmap"
    (src / "sparse").mkdir(parents=True)
    for name, data in fx["sparse"].items():
        (src / "sparse" / name).write_bytes(base64.b64decode(data))
    (src / "images").mkdir()
    for name in fx["image_names"]:
        (src / "images" / name).write_bytes(b"JPEG placeholder " + name.encode())
    dst = tmp_path / "dense"
    a = fx["args"]
    colmap.process_scene(str(src), str(dst), fx["model_ext"], a["max_d"], a["interval_scale"], a["theta0"],
                         a["top_k"], a["min_shared"], log=lambda *x: None)
    got = {os.path.relpath(p, dst): open(p).read()
           for p in glob.glob(str(dst / "**" / "*"), recursive=True)
           if os.path.isfile(p) and "images" not in os.path.relpath(p, dst)}
    assert sorted(got) == sorted(fx["expected"])
    for name, text in fx["expected"].items():
        assert got[name] == text, name


def test_fixtures_present_and_nontrivial():
    assert len(FIXTURES) >= 4
    nonempty = 0
    for path in FIXTURES:
        fx = json.load(open(path))
        lines = fx["expected"]["pair.txt"].split("\n")
        nonempty += sum(1 for ln in lines[2::2] if ln.strip() and int(ln.split()[0]) > 0)
    assert nonempty > 20
