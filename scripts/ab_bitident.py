"""A/B helper (GPU box): run RunPatchMatch on SPHERE scenes with one library build (ACMMP_LIB) and save the
planes / costs, or compare the saved outputs of several builds bit for bit.

  python scripts/ab_bitident.py run OUT.npz [--math fast|exact]     (in a process with ACMMP_LIB set)
  python scripts/ab_bitident.py cmp A.npz B.npz ...
Scenes: the bench metric (2000x1500 V=4), 3200x1600 V=15 (C3 size, view-chunked), a small 640x320 V=4 and the C2
pinhole rig (1600x1200 V=10)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "acmmp-spherical_amd"))
import numpy as np  # noqa: E402

CASES = [(2000, 1500, 4, 1235), (3200, 1600, 15, 7), (640, 320, 4, 3), (1600, 1200, 10, 9)]


def run(out, math):
    from acmmp import capi, scene, types
    res = {}
    for (W, H, V, seed) in CASES:
        sc = (scene.pinhole_scene(W, H, n_src=V, seed=seed) if (W, H, V) == (1600, 1200, 10)
              else scene.sphere_scene(W, H, n_src=V, seed=seed))
        c0 = sc.cameras[0]
        p = types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                                 depth_max=float(c0["depth_max"]) * 1.2)
        with capi.Context(0) as ctx:
            ctx.set_math(math)
            ctx.set_params(p)
            ctx.upload_views(sc.images, sc.cameras)
            ctx.run_patchmatch(11)
            pl, co = ctx.download()
        res[f"planes_{W}x{H}_{V}"] = pl
        res[f"costs_{W}x{H}_{V}"] = co
        print(os.path.basename(os.environ.get("ACMMP_LIB", "libacmmp.so")), W, H, V, "done", flush=True)
    np.savez(out, **res)


def cmp(paths):
    base = np.load(paths[0])
    ok = True
    for p in paths[1:]:
        other = np.load(p)
        for k in base.files:
            a, b = base[k].view(np.uint32), other[k].view(np.uint32)
            d = int((a != b).sum())
            ok &= d == 0
            print(os.path.basename(p), k, "differing words:", d, "of", a.size)
    print("BITIDENT" if ok else "DIFFER")
    return 0 if ok else 1


if __name__ == "__main__":
    if sys.argv[1] == "run":
        math = sys.argv[4] if len(sys.argv) > 4 and sys.argv[3] == "--math" else "fast"
        run(sys.argv[2], math)
    else:
        sys.exit(cmp(sys.argv[2:]))
