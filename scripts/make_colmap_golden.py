"""Generate tests/golden/colmap_*.json: the reference converter's own outputs on synthetic sparse models.

Runs the reference's colmap2mvsnet_acm.py (`process_scene`, :249-406) from /root/reference -- in this
container only; the GPU box has no reference -- on seeded synthetic COLMAP models (tests/test_colmap.py's
generator) in both encodings, and stores the inputs (the sparse model files) and the outputs the
reference writes (cams/*_cam.txt, pair.txt) as data.  tests/test_colmap_golden.py replays the inputs
through acmmp.colmap and requires byte-identical files.

The script imports cv2 at module level (:26) but calls it only to re-encode non-.jpg images (:404);
OpenCV is not installed here, so a placeholder module is registered under that name whose every
attribute access raises: nothing of OpenCV is imitated, and every case uses .jpg inputs, so the
reference's own code is what runs.  Re-run with `python scripts/make_colmap_golden.py`.
"""
import argparse
import base64
import importlib.util
import json
import os
import sys
import tempfile
import types as pytypes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/colmap2mvsnet_acm.py"
sys.path.insert(0, os.path.join(REPO, "acmmp-spherical_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

from acmmp import colmap  # noqa: E402
from test_colmap import synthetic_model  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")

CASES = [
    # name, model kwargs, encoding, converter arguments
    ("pinhole_txt", dict(n_images=8, n_points=150, seed=3), ".txt",
     dict(max_d=192, interval_scale=1.0, theta0=1.0, top_k=4, min_shared=5)),
    ("sphere_bin", dict(n_images=8, n_points=150, sphere=True, seed=4), ".bin",
     dict(max_d=0, interval_scale=1.0, theta0=1.0, top_k=3, min_shared=5)),
    ("pinhole_theta_bin", dict(n_images=10, n_points=150, seed=5), ".bin",
     dict(max_d=0, interval_scale=0.5, theta0=20.0, top_k=5, min_shared=8)),
    ("sphere_txt_topk", dict(n_images=9, n_points=120, sphere=True, seed=6), ".txt",
     dict(max_d=128, interval_scale=2.0, theta0=0.5, top_k=8, min_shared=3)),
]


class _Unavailable(pytypes.ModuleType):
    def __getattr__(self, name):
        raise RuntimeError(f"cv2.{name} called: OpenCV is not available to the golden generator")


def load_reference():
    sys.modules.setdefault("cv2", _Unavailable("cv2"))
    spec = importlib.util.spec_from_file_location("colmap2mvsnet_acm", REF)
    mod = importlib.util.module_from_spec(spec)
    sys.modules["colmap2mvsnet_acm"] = mod
    spec.loader.exec_module(mod)
    return mod


def files_under(root):
    out = {}
    for dp, _, fs in os.walk(root):
        for f in sorted(fs):
            p = os.path.join(dp, f)
            out[os.path.relpath(p, root)] = open(p, "rb").read()
    return out


def main():
    ref = load_reference()
    os.makedirs(OUT, exist_ok=True)
    for name, mkw, ext, args in CASES:
        cams, imgs, pts = synthetic_model(**mkw)
        with tempfile.TemporaryDirectory() as tmp:
            src = os.path.join(tmp, "colmap")
            (colmap.write_model_text if ext == ".txt" else colmap.write_model_binary)(
                os.path.join(src, "sparse"), cams, imgs, pts)
            os.makedirs(os.path.join(src, "images"))
            for im in imgs.values():
                with open(os.path.join(src, "images", im.name), "wb") as f:
                    f.write(b"JPEG placeholder " + im.name.encode())
            dst = os.path.join(tmp, "dense")
            os.makedirs(dst)
            ref.process_scene(argparse.Namespace(dense_folder=src, save_folder=dst, model_ext=ext, chunksize=512,
                                                 **args))
            inputs = files_under(os.path.join(src, "sparse"))
            outputs = {k: v for k, v in files_under(dst).items() if not k.startswith("images")}
        fixture = {
            "generator": "scripts/make_colmap_golden.py (reference colmap2mvsnet_acm.py process_scene)",
            "model_ext": ext, "args": args,
            "image_names": [imgs[k].name for k in sorted(imgs)],
            "sparse": {k: base64.b64encode(v).decode() for k, v in inputs.items()},
            "expected": {k: v.decode() for k, v in outputs.items()},
        }
        path = os.path.join(OUT, f"colmap_{name}.json")
        with open(path, "w") as f:
            json.dump(fixture, f, indent=0, sort_keys=True)
        print(path, len(outputs), "files", os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
