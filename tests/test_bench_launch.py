"""bench.py's launch contract, on the CPU: `--gpus N` is
authoritative -- from plain `python` it starts N rank processes with the
env:// rendezvous variables (the driver's `python bench.py --gpus N` shape),
under torchrun it must agree with WORLD_SIZE -- and the launcher reports the
first failing rank.  The rank script here is a stand-in that records its
environment (the real ranks need a GPU)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

RANK_SCRIPT = """
import json, os, sys, time
out = sys.argv[1]
keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
        "EWARP_BENCH_LAUNCHER", "EWARP_BENCH_CPU_JSON"]
rec = {k: os.environ.get(k) for k in keys}
if rec["EWARP_BENCH_CPU_JSON"]:
    rec["cpu"] = json.load(open(rec["EWARP_BENCH_CPU_JSON"]))
rec["argv"] = sys.argv[2:]
with open(os.path.join(out, "rank%s.json" % rec["RANK"]), "w") as fh:
    json.dump(rec, fh)
if "--fail-rank" in sys.argv and sys.argv[sys.argv.index("--fail-rank") + 1] == rec["RANK"]:
    sys.exit(3)
if "--fail-rank" in sys.argv:
    time.sleep(120)       # the launcher must stop this one
"""


def test_rank_environments():
    envs = bench.rank_environments(2, 29512, base={"PATH": "/bin", bench.CPU_JSON_ENV: "stale"})
    assert len(envs) == 2
    for r, e in enumerate(envs):
        assert e["RANK"] == e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "2"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29512"
        assert e[bench.LAUNCHER_ENV] == "1" and e["PATH"] == "/bin"
        assert bench.CPU_JSON_ENV not in e


def test_resolve_world():
    assert bench.resolve_world(None, {}) == (1, False)
    assert bench.resolve_world(1, {}) == (1, False)
    assert bench.resolve_world(2, {}) == (2, True)
    assert bench.resolve_world(8, {}) == (8, True)
    assert bench.resolve_world(None, {"WORLD_SIZE": "4"}) == (4, False)
    assert bench.resolve_world(4, {"WORLD_SIZE": "4"}) == (4, False)
    with pytest.raises(SystemExit):
        bench.resolve_world(2, {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        bench.resolve_world(0, {})


def test_launch_two_ranks(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    cpu = {"value": 123.0, "cores": 16}
    rc = bench.launch(2, [str(tmp_path), "--gpus", "2"], cpu=cpu, script=str(script))
    assert rc == 0
    recs = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(2)]
    for r, rec in enumerate(recs):
        assert rec["RANK"] == rec["LOCAL_RANK"] == str(r)
        assert rec["WORLD_SIZE"] == "2" and rec["MASTER_ADDR"] == "127.0.0.1"
        assert rec["EWARP_BENCH_LAUNCHER"] == "1"
        assert rec["argv"] == ["--gpus", "2"]
    assert recs[0]["MASTER_PORT"] == recs[1]["MASTER_PORT"]
    assert recs[0]["cpu"] == cpu                  # the launcher's CPU baseline reaches rank 0 only
    assert recs[1]["EWARP_BENCH_CPU_JSON"] is None
    assert not os.path.exists(recs[0]["EWARP_BENCH_CPU_JSON"])   # removed after the run


def test_launch_stops_on_failing_rank(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    import time
    t0 = time.time()
    rc = bench.launch(3, [str(tmp_path), "--fail-rank", "1"], script=str(script))
    assert rc == 3
    assert time.time() - t0 < 60                  # the sleeping ranks were terminated


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_verify_on_by_default_with_ranks():
    """a plain multi-rank `bench.py --gpus N` verifies by
    default (the driver passes no flag); --no-verify / --verify override."""
    assert bench.verify_default(None, 1) is False
    assert bench.verify_default(None, 2) is True and bench.verify_default(None, 8) is True
    assert bench.verify_default(False, 8) is False and bench.verify_default(True, 1) is True


def test_run_problems():
    """Rank 0 exits non-zero when two ranks sit on one device without
    --same-device, or the verify block is missing / failed."""
    a = {"index": 0, "pci_bus_id": "0000:05:00.0", "uuid": "u0"}
    b = {"index": 1, "pci_bus_id": "0000:15:00.0", "uuid": "u1"}
    ok = {"samples": 256, "max_err_over_strict": 1e-4, "inf_pattern_equal": True}
    assert bench.run_problems([a, b], False, ok, True) == []
    assert bench.run_problems([a, dict(a, index=1)], False, ok, True)            # one device twice
    assert bench.run_problems([a, dict(a, index=1)], True, ok, True) == []       # the rehearsal
    assert bench.run_problems([a, b], False, None, True)                         # verify missing
    assert bench.run_problems([a, b], False, dict(ok, max_err_over_strict=2.0), True)
    assert bench.run_problems([a, b], False, dict(ok, inf_pattern_equal=False), True)
    assert bench.run_problems([a], False, None, False) == []


def test_bench_parser_verify_flags(monkeypatch):
    """The CLI carries both flags; a rank of a plain `--gpus 2` run gets
    args.verify True (main() resolves it before anything touches a GPU)."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert '"--no-verify"' in src and "args.verify = verify_default(args.verify, world)" in src
    assert 'rec["verify"] = verify' in src and "sys.exit(3)" in src
