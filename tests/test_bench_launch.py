"""bench.py --gpus N launches its own ranks (CPU; no GPU touched).

The driver runs `python bench.py --gpus N` for the N=1 line and, for the scaling curve, either the same
command or a torch.distributed.run launch of it.  Run directly with N > 1, bench.py starts N gloo ranks
itself (torch.distributed.run child, rendezvous on 127.0.0.1); `--dry-run` stops every rank right after
the rendezvous, so the plumbing is checked without a device.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=ROOT)


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_gpus2_spawns_two_gloo_ranks():
    r = _bench("--gpus", "2", "--dry-run")
    assert r.returncode == 0, r.stderr[-2000:]
    line = _json_line(r.stdout)
    assert line["ranks"] == 2 and line["rank_ids"] == [0, 1]
    assert line["processes"] == 2 and line["backend"] == "gloo" and line["gpus"] == 2


def test_gpus3_pipeline_mode_spawns_three_ranks():
    r = _bench("--gpus", "3", "--mode", "pipeline", "--dry-run")
    assert r.returncode == 0, r.stderr[-2000:]
    assert _json_line(r.stdout)["rank_ids"] == [0, 1, 2]


def test_gpus1_dry_run_single_process():
    r = _bench("--dry-run")
    assert r.returncode == 0, r.stderr[-2000:]
    line = _json_line(r.stdout)
    assert line["ranks"] == 1 and line["backend"] is None


def test_refuses_more_ranks_than_gpus():
    # this container has no GPU: asking for 2 must fail loudly, not run one rank and report it as 2
    r = _bench("--gpus", "2", "--steps", "1", "--warmup", "0")
    assert r.returncode == 2
    assert "refusing" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_launcher_world_mismatch_is_an_error():
    r = _bench("--gpus", "4", "--dry-run", env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "launcher started 1" in r.stderr


def test_abandoned_extra_exits_nonzero():
    """A guarded extra abandoned at its deadline (a hung first RCCL run) prints the line with the error and
    then exits non-zero on every rank, so the driver does not read the hang as success."""
    r = _bench("--gpus", "2", "--dry-run", env={"ACMMP_BENCH_SELFTEST_ABANDON": "1"})
    assert r.returncode != 0, r.stderr[-2000:]
    line = _json_line(r.stdout)
    assert line["ranks"] == 2 and "abandoned" in line["extra"]["error"]
    r1 = _bench("--dry-run", env={"ACMMP_BENCH_SELFTEST_ABANDON": "1"})
    assert r1.returncode == 3


def test_visible_gpus_counts_without_hip():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    n = bench.visible_gpus()
    assert n >= 0
    os.environ["HIP_VISIBLE_DEVICES"] = ""
    try:
        assert bench.visible_gpus() == 0
    finally:
        del os.environ["HIP_VISIBLE_DEVICES"]
    assert "torch" not in bench.visible_gpus.__code__.co_names


def test_multi_rank_extras_are_guarded():
    """The first runs of the RCCL extras (depth_exchange, band_split) cannot cost the headline line: an
    exception is reported in the line, and a hang is abandoned at the deadline."""
    import importlib.util
    import time
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)

    def boom():
        raise RuntimeError("rccl said no")
    r, abandoned = bench.guarded(boom, 5)
    assert not abandoned and "rccl said no" in r["error"]
    r, abandoned = bench.guarded(lambda x: {"ok": x}, 5, 7)
    assert r == {"ok": 7} and not abandoned
    t0 = time.perf_counter()
    r, abandoned = bench.guarded(time.sleep, 0.5, 30)
    assert abandoned and "abandoned" in r["error"] and time.perf_counter() - t0 < 5
