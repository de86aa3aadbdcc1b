"""The reference's on-disk formats and multi-scale schedule (acmmp/io.py)."""
import os

import numpy as np

from acmmp import io, scene, types


def test_dmb_roundtrip(tmp_path):
    d = np.random.default_rng(0).normal(size=(7, 5)).astype(np.float32)
    n = np.random.default_rng(1).normal(size=(7, 5, 3)).astype(np.float32)
    io.write_dmb(str(tmp_path / "d.dmb"), d)
    io.write_dmb(str(tmp_path / "n.dmb"), n)
    raw = open(tmp_path / "d.dmb", "rb").read()
    assert np.frombuffer(raw[:16], "<i4").tolist() == [1, 7, 5, 1]      # ACMMP.cpp:403-411
    assert np.array_equal(io.read_dmb(str(tmp_path / "d.dmb")), d)
    assert np.array_equal(io.read_dmb(str(tmp_path / "n.dmb")), n)
    assert io.read_dmb(str(tmp_path / "missing.dmb")) is None
    (tmp_path / "bad.dmb").write_bytes(np.array([2, 1, 1, 1], "<i4").tobytes())
    assert io.read_dmb(str(tmp_path / "bad.dmb")) is None               # type != 1 -> -1


def test_read_camera_sphere_and_pinhole_quirk(tmp_path):
    sc = scene.sphere_scene(64, 32, n_src=1, seed=0)
    io.write_camera(str(tmp_path / "s.txt"), sc.cameras[1], depth_interval=0.1, n_planes=192)
    c = io.read_camera(str(tmp_path / "s.txt"))
    assert int(c["model"]) == types.SPHERE
    assert np.allclose(c["params"][:3], sc.cameras[1]["params"][:3])
    assert np.allclose(c["R"], sc.cameras[1]["R"]) and np.allclose(c["t"], sc.cameras[1]["t"])
    assert np.float32(c["depth_max"]) == np.float32(sc.cameras[1]["depth_max"])
    # PINHOLE: the converter writes `d0 dint N dmax`; ReadCamera keeps the 2nd token (ACMMP.cpp:205)
    pc = scene.pinhole_scene(32, 24, n_src=1, seed=0).cameras[0]
    io.write_camera(str(tmp_path / "p.txt"), pc, depth_interval=0.25, n_planes=192)
    c = io.read_camera(str(tmp_path / "p.txt"))
    assert int(c["model"]) == types.PINHOLE
    assert np.allclose(c["K"], pc["K"])
    assert np.float32(c["depth_min"]) == np.float32(pc["depth_min"])
    assert np.float32(c["depth_max"]) == np.float32(0.25)


def test_pair_list_drops_nonpositive_scores(tmp_path):
    io.write_pair_list(str(tmp_path), [(0, [(1, 0.5), (2, 0.0), (3, -1.0), (4, 2.0)]), (1, [(0, 1.0)])])
    ps = io.read_pair_list(str(tmp_path))
    assert [p.ref_image_id for p in ps] == [0, 1]
    assert ps[0].src_image_ids == [1, 4] and ps[1].src_image_ids == [0]


def test_multiscale_settings_match_survey_table():
    """main.cpp:35-71 + :417-425."""
    cases = {(1500, 2000): [1000, 2000], (1200, 1600): [800, 1600], (4000, 6000): [800, 1600, 3200],
             (2048, 4096): [800, 1600, 3200], (1080, 1920): [960, 1920]}
    for (rows, cols), want in cases.items():
        ps = [io.Problem(0)]
        k = io.compute_multiscale_settings(ps, {0: (rows, cols)})
        assert [s[0] for s in io.scale_schedule(ps, k)] == want
