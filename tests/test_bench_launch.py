"""bench.py's own multi-rank launcher (the driver runs `python bench.py --gpus N`
without torchrun): N rank processes with RANK / WORLD_SIZE / MASTER_* on
127.0.0.1, rank 0's JSON line forwarded, a failing rank fails the run.  CPU only:
SPE_BENCH_LAUNCH_DRYRUN makes every rank join a gloo group and all-reduce
instead of touching a GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e["SPE_BENCH_LAUNCH_DRYRUN"] = "1"
    e.update(kw)
    return e


def test_gpus_two_spawns_two_gloo_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--no-side"], env=_env(), capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["rank_sum"] == 3.0   # ranks 1 + 2: both joined one group


def test_gpus_three_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3"], env=_env(), capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert out["n_gpus"] == 3 and out["rank_sum"] == 6.0


def test_world_size_must_match_gpus():
    """Under torchrun, --gpus N must agree with WORLD_SIZE (no silent one-GPU run)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                                MASTER_PORT="29555"), capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE" in (r.stdout + r.stderr)


def test_failing_rank_fails_the_run():
    # a rank that dies (here: an unknown config raises SystemExit in every rank) must
    # make the launcher exit non-zero instead of printing a line
    e = _env()
    e.pop("SPE_BENCH_LAUNCH_DRYRUN")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--config", "nonexistent"], env=e,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]
