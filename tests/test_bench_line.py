"""bench.py's final stdout line must be parseable from the driver's stdout tail
(a 22.6-KB line with every side config's full record was cut and
BENCH_r05 recorded `parsed: null`).  The line is built here from the round-5
full record (profiles/r05_bench_default_with_side_configs.json, every side
config included) through the same emit() the bench calls, in a child process,
and the LAST stdout line is parsed: the headline fields, `roofline` and
`cpu_baseline` survive whole, and the line stays under bench.LINE_MAX_BYTES."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FULL = os.path.join(ROOT, "profiles", "r05_bench_default_with_side_configs.json")

HEADLINE = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def _emit_in_child(tmp_path, record):
    src = tmp_path / "rec.json"
    src.write_text(json.dumps(record))
    code = ("import json, sys; sys.path.insert(0, %r); import bench; "
            "bench.emit(json.load(open(%r)), '_linetest')" % (ROOT, str(src)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    return r


def test_default_line_with_side_configs_parses_and_fits(tmp_path):
    sys.path.insert(0, ROOT)
    import bench
    record = json.load(open(FULL))
    assert len(json.dumps(record)) > 20000   # the round-5 line the driver could not parse
    r = _emit_in_child(tmp_path, record)
    last = r.stdout.rstrip("\n").splitlines()[-1]
    assert len(last.encode()) <= bench.LINE_MAX_BYTES
    out = json.loads(last)
    for k in HEADLINE:
        assert k in out, k
        assert out[k] == record[k], k   # headline, roofline and cpu_baseline unchanged
    assert out["roofline"]["frac"] > 0 and out["cpu_baseline"]["value"] > 0
    # every side config keeps its value and (for tables) its roofline fraction
    assert set(out["side_configs"]) == set(record["side_configs"])
    for name, v in record["side_configs"].items():
        s = out["side_configs"][name]
        assert s["value"] == v["value"], name
        if (v.get("roofline") or {}).get("frac") is not None:
            assert s["frac"] == v["roofline"]["frac"], name
    assert out["side_configs"]["c3_exact"]["vs_default_build"]["route_mismatch"] == 0
    # the full record is kept in the file the line names, and the headline is echoed on stderr
    full = os.path.join(ROOT, out["full_record"])
    try:
        assert json.load(open(full)) == record
    finally:
        os.remove(full)
    assert "[bench] headline: %s" % record["value"] in r.stderr


def test_oversized_side_configs_still_fit(tmp_path):
    """Even twenty side configs with long error tails leave a parseable line."""
    sys.path.insert(0, ROOT)
    import bench
    record = json.load(open(FULL))
    side = dict(record["side_configs"])
    for i in range(20):
        side[f"extra{i}"] = {"error": "exit status 1", "tail": "x" * 600, "wall_s": 1.0}
    record["side_configs"] = side
    r = _emit_in_child(tmp_path, record)
    last = r.stdout.rstrip("\n").splitlines()[-1]
    assert len(last.encode()) <= bench.LINE_MAX_BYTES
    out = json.loads(last)
    assert out["value"] == record["value"] and out["roofline"] == record["roofline"]
    os.remove(os.path.join(ROOT, out["full_record"]))


def test_short_line_printed_whole(tmp_path):
    record = {"metric": "m", "value": 1.0, "unit": "sources/s", "n_gpus": 1, "roofline": {"frac": 0.1},
              "cpu_baseline": {"value": 2.0}}
    r = _emit_in_child(tmp_path, record)
    assert json.loads(r.stdout.strip().splitlines()[-1]) == record
