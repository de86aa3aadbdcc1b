"""The oracle's control logic against a second restatement written from the reference source
(tests/np_propagation.py, scalar float32 Python): RandomInitialization, CheckerboardPropagation
and PlaneHypothesisRefinement (ACMMP.cu:673-1325), per pixel and per half-sweep.

Compared bit for bit after init and after every half-sweep: planes, costs, selected_views, and for
every pixel the half-sweep updated (oracle or_trace): the eight picked neighbour positions (-1 where
flag[d] is false), the per-view weights of the 15 draws, the aggregated costs, FindMinCostIndex /
FindMaxCostIndex, the hypothesis accepted into plane_hypotheses_now, temp_selected_views and the
RNG draw counter before/after.  Both sides take the bilateral NCC, the geometric cost and the
elementary functions from the same pinned definitions (np_propagation.py docstring), so a
disagreement is a disagreement about the decision logic or its arithmetic order.

Scenes: tiny pinhole and SPHERE rigs with V in {1, 4, 15, 20, 32} (the reference's maximum,
cost_vector[32], ACMMP.cu:522,957,1153), plus geometric-consistency, planar-prior and hierarchy
(pre_costs gate) passes.  No GPU.
"""
import numpy as np
import pytest

import np_propagation as npp
from acmmp import scene, types


def params_for(sc, **kw):
    c0 = sc.cameras[0]
    return types.default_params(num_images=len(sc.images), depth_min=float(c0["depth_min"]) * 0.6,
                                depth_max=float(c0["depth_max"]) * 1.2, **kw)


def make(kind, W, H, V, seed):
    if kind == "pinhole":
        return scene.pinhole_scene(W, H, n_src=V, seed=seed, n_waves=24)
    return scene.sphere_scene(W, H, n_src=V, seed=seed, n_waves=24)


TRACE_FIELDS = ("pos", "view_weights", "final_costs", "cost_now", "min_idx", "max_idx", "accepted",
                "temp_selected_views", "draws_before", "draws_after")


def _eq(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype.kind == "f":
        return np.array_equal(a.view(np.uint32 if a.dtype == np.float32 else np.uint64),
                              b.view(np.uint32 if b.dtype == np.float32 else np.uint64)) or \
            np.array_equal(a, b, equal_nan=True)
    return np.array_equal(a, b)


def compare_run(oracle_mod, sc, p, seed, n_half_sweeps, prior=None, masks=None, depths=None, state=None,
                pre_costs=None, scaled=None):
    H, W = sc.images[0].shape
    prob = oracle_mod.Problem(sc.images, sc.cameras, p, depths=depths, prior_planes=prior, plane_masks=masks,
                              scaled_planes=scaled)
    R = npp.Restatement(sc.images, sc.cameras, p, seed,
                        ncc=lambda v, x, y, pl: oracle_mod.ncc(prob, v, x, y, pl),
                        geom=lambda v, x, y, pl: oracle_mod.geom_cost(prob, v, x, y, pl),
                        detmath=oracle_mod.detmath, prior=prior, masks=masks)
    planes = np.zeros((H, W, 4), np.float32) if state is None else state[0].copy()
    costs = np.zeros((H, W), np.float32) if state is None else state[1].copy()
    pre = np.zeros((H, W), np.float32) if pre_costs is None else pre_costs.copy()
    sel = np.zeros((H, W), np.uint32)
    draws = np.zeros((H, W), np.int64)
    kw = dict(planes=None if state is None else state[0], costs=None if state is None else state[1],
              pre_costs=pre_costs, do_post=False, nthreads=4)
    R.init(planes, costs, sel, draws, scaled=scaled)
    stats = {"accepted_neighbour": 0, "accepted_refine": 0, "pixels": 0}
    for k in range(n_half_sweeps + 1):
        if k > 0:
            trace = np.zeros((H, W), oracle_mod.TRACE_DTYPE)
            trace["min_idx"] = -2
            R.half_sweep(planes, costs, pre, sel, draws, colour=(k - 1) & 1, it=(k - 1) // 2, trace=trace)
        o = oracle_mod.run_patchmatch_traced(prob, seed, n_half_sweeps=k, **kw)
        where = f"after {'init' if k == 0 else f'half-sweep {k}'}"
        assert _eq(planes, o["planes"]), f"planes differ {where}: {np.argwhere(planes != o['planes'])[:5]}"
        assert _eq(costs, o["costs"]), f"costs differ {where}"
        assert np.array_equal(sel, o["selected_views"]), f"selected_views differ {where}"
        if k == 0:
            continue
        upd = trace["min_idx"] != -2
        assert upd.sum() > 0
        ot = o["trace"]
        for f in TRACE_FIELDS:
            assert _eq(trace[f][upd], ot[f][upd]), f"trace field {f} differs {where}"
        acc = trace["accepted"][upd]
        stats["accepted_neighbour"] += int(((acc >= 0) & (acc < 8)).sum())
        stats["accepted_refine"] += int((acc >= 9).sum())
        stats["pixels"] += int(upd.sum())
    return stats


CASES = [("pinhole", 24, 20, 1), ("pinhole", 24, 20, 4), ("pinhole", 20, 16, 15), ("pinhole", 20, 14, 20),
         ("pinhole", 16, 14, 32), ("sphere", 32, 16, 1), ("sphere", 32, 16, 4), ("sphere", 24, 12, 15),
         ("sphere", 20, 12, 32)]


@pytest.mark.parametrize("kind,W,H,V", CASES, ids=[f"{k}-{w}x{h}-v{v}" for k, w, h, v in CASES])
def test_random_init_and_half_sweeps_match_second_restatement(oracle_mod, kind, W, H, V):
    sc = make(kind, W, H, V, seed=V + W)
    p = params_for(sc)
    n_hs = 3 if V <= 15 else 2
    stats = compare_run(oracle_mod, sc, p, seed=1000 + V, n_half_sweeps=n_hs)
    # the comparison exercised both kinds of update
    assert stats["accepted_neighbour"] > 0 and stats["accepted_refine"] > 0, stats


def _first_pass(oracle_mod, sc, seed=3):
    p0 = params_for(sc)
    return oracle_mod.run_patchmatch(oracle_mod.Problem(sc.images, sc.cameras, p0), seed=seed, nthreads=4)


@pytest.mark.parametrize("kind,V", [("pinhole", 4), ("sphere", 3)])
def test_geom_pass_matches_second_restatement(oracle_mod, kind, V):
    """Reuse branch (ACMMP.cu:780-793) + geometric-consistency aggregation (:1214-1216, :1236-1240,
    :888-892) from a first pass's (world-frame normal, depth) state."""
    sc = make(kind, 24, 16, V, seed=70 + V)
    first = _first_pass(oracle_mod, sc)
    rng = np.random.default_rng(V)
    d0 = first["planes"][..., 3]
    depths = [d0] + [(d0 * rng.uniform(0.97, 1.03, d0.shape)).astype(np.float32) for _ in range(V)]
    pg = params_for(sc, geom_consistency=1, max_iterations=2)
    compare_run(oracle_mod, sc, pg, seed=11, n_half_sweeps=2, depths=depths,
                state=(first["planes"], first["costs"]))


@pytest.mark.parametrize("kind", ["pinhole", "sphere"])
def test_planar_prior_pass_matches_second_restatement(oracle_mod, kind):
    """Planar-prior init branch (:690-711), restricted-cost selection (:1247-1299) and prior-restricted
    refinement (:823-836, :908-925) with geometric consistency on (the ProcessProblem order)."""
    sc = make(kind, 24, 16, 2, seed=90)
    H, W = 16, 24
    first = _first_pass(oracle_mod, sc)
    rng = np.random.default_rng(7)
    prior = np.zeros((H, W, 4), np.float32)
    prior[..., 2] = -1.0
    prior[..., :3] += rng.normal(0, 0.1, (H, W, 3)).astype(np.float32)
    prior[..., :3] /= np.linalg.norm(prior[..., :3], axis=-1, keepdims=True)
    prior[..., 3] = (sc.gt_depth * rng.uniform(0.95, 1.05, (H, W))).astype(np.float32)
    masks = ((rng.uniform(size=(H, W)) < 0.7) * rng.integers(1, 9, (H, W))).astype(np.uint32)
    d0 = first["planes"][..., 3]
    depths = [d0] + [(d0 * rng.uniform(0.97, 1.03, d0.shape)).astype(np.float32) for _ in range(2)]
    pp = params_for(sc, geom_consistency=1, planar_prior=1, max_iterations=2)
    state_costs = first["costs"].copy()
    state_costs[::3, ::2] = 0.05                           # some pixels below the 0.1 init gate
    compare_run(oracle_mod, sc, pp, seed=12, n_half_sweeps=2, prior=prior, masks=masks, depths=depths,
                state=(first["planes"], state_costs))


def test_hierarchy_gate_matches_second_restatement(oracle_mod):
    """Hierarchy reuse init (:784-786 with scaled_plane_hypotheses) and the pre_costs gate
    (:1315-1320): a refined hypothesis is kept only when it beats pre_costs - 0.1."""
    sc = make("pinhole", 24, 16, 3, seed=110)
    H, W = 16, 24
    first = _first_pass(oracle_mod, sc)
    rng = np.random.default_rng(9)
    scaled = first["planes"].copy()
    pre = rng.uniform(0.0, 1.0, (H, W)).astype(np.float32)
    ph = params_for(sc, hierarchy=1)
    compare_run(oracle_mod, sc, ph, seed=13, n_half_sweeps=2, scaled=scaled, pre_costs=pre,
                state=(first["planes"], first["costs"]))


def test_rng_restatement_matches_oracle_stream(oracle_mod):
    """The restated Philox stream equals the oracle's per-pixel draws (which Random123 vectors pin)."""
    for seed, sub in [(0, 0), (1234, 77), (2 ** 40 + 5, 123456), (99, 2 ** 20 + 3)]:
        rs = npp.PixelRng(seed, sub)
        for n in range(11):
            assert npp.F(rs.uniform()) == npp.F(oracle_mod.uniform_draw(seed, sub, n))


def test_fma_emulation_is_correctly_rounded():
    rng = np.random.default_rng(0)
    a = rng.normal(size=2000).astype(np.float32)
    b = rng.normal(size=2000).astype(np.float32)
    c = (rng.normal(size=2000) * 10.0 ** rng.integers(-8, 8, 2000)).astype(np.float32)
    from fractions import Fraction
    for x, y, z in zip(a[:300], b[:300], c[:300]):
        exact = Fraction(float(x)) * Fraction(float(y)) + Fraction(float(z))
        r = npp.fma(x, y, z)
        lo, hi = np.nextafter(r, np.float32(-np.inf)), np.nextafter(r, np.float32(np.inf))
        err = abs(Fraction(float(r)) - exact)
        assert err <= abs(Fraction(float(lo)) - exact) and err <= abs(Fraction(float(hi)) - exact)
    # a constructed midpoint case: 1 + 2^-24 (a binary32 tie) plus a tiny product decides the direction
    assert npp.fma(np.float32(2.0 ** -30), np.float32(2.0 ** -30), np.float32(1.0) + np.float32(0)) == np.float32(1.0)
    tie_up = npp.fma(np.float32(1.0 + 2.0 ** -23), np.float32(1.0 + 2.0 ** -23), np.float32(0.0))
    assert tie_up == np.float32((1.0 + 2.0 ** -23) ** 2)
