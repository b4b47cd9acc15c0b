"""bench.py's multi-rank contract on the CPU: ``--gpus N`` without a launcher spawns N
rank processes itself, the JSON's n_gpus / world_size come from the process group, a mismatch with
WORLD_SIZE and an RCCL request for more GPUs than visible both fail loudly."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
TINY = ["--device", "cpu", "--model", "raftstereo-realtime", "--per-gpu-batch", "1", "--height", "128",
        "--width", "160", "--iters", "1", "--steps", "2", "--warmup", "1"]


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env)
    return subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], env=e, capture_output=True,
                          text=True, timeout=600)


def _json(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_self_launch_two_ranks_gloo():
    r = _run(["--gpus", "2", *TINY], SA_DIST_BACKEND="gloo")
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json(r.stdout)
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2
    assert rec["config"]["parallelism"] == "dp2" and rec["config"]["global_batch"] == 2
    assert sorted(x["rank"] for x in rec["ranks"]) == [0, 1]
    assert rec["allgather_ms"] is not None and rec["value"] > 0
    assert "oracle" in rec["engine"]


def test_single_rank_cpu():
    r = _run(["--gpus", "1", *TINY])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json(r.stdout)
    assert rec["n_gpus"] == 1 and rec["config"]["parallelism"] == "dp1"


def test_more_gpus_than_visible_fails():
    r = _run(["--gpus", "9", "--steps", "1", "--warmup", "0"], SA_DIST_BACKEND="nccl")
    assert r.returncode != 0
    assert "GPU" in r.stderr


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "4", *TINY], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_scale_report_cpu(tmp_path):
    out = tmp_path / "scale.md"
    e = dict(os.environ, SA_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "scale_report.py"), "--sizes", "1,2", "--out", str(out),
                        *TINY], env=e, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rows = json.loads(out.with_suffix(".json").read_text())
    assert [x["n_gpus"] for x in rows] == [1, 2]
    assert "| 2 |" in out.read_text()
