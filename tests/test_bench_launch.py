"""CPU: bench.py's launcher and distributed plumbing without a GPU.  `bench.py --gpus 2`
with no torch.distributed environment starts torch.distributed.run itself (before any GPU
call); --backend gloo --dry-run then runs the shard plan, the shared chromosome queue over
the default store (the C5 leg's load balancing, its input produced per pulled ticket) and the
(score, p) track gathers (all-gather and gather to rank 0)."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def test_bench_spawns_ranks_and_gathers():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MASTER_ADDR"] = "127.0.0.1"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--backend", "gloo", "--dry-run",
                        "--c45-chroms", "4"], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = lines[0]
    assert out["dry_run"] and out["n_gpus"] == 2 and out["gather_ok"] and out["gather_to_0_ok"]
    assert sum(out["queue_per_rank"]) == 8 and out["static_per_rank"] == [4, 4]
    # the C5 queue moves the input with the ticket: only pulled chromosomes are made, two at a time
    assert out["materialised_only_pulled"] and out["max_live_inputs"] <= 2


def test_bench_dry_run_walks_every_leg_at_four_ranks():
    """Round-4 hang guard: the bench's legs in their real order at world size 4 (gloo, device
    work stubbed) -- the FET timed steps and track gather, C3, the C4 static plan and gather,
    the C5 ticket queue, its all-reduce and gather -- must bring every rank to the final
    barrier, and the C5 queue must hand each chromosome to exactly one rank."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MASTER_ADDR"] = "127.0.0.1"
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "4", "--backend", "gloo", "--dry-run",
                        "--nsnp", "3000", "--nchrom", "2", "--c45-chroms", "2", "--steps", "2", "--warmup", "1",
                        "--css-steps", "2", "--c45-steps", "2", "--trace-hang", "60"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = lines[0]
    assert out["dry_run"] and out["n_gpus"] == 4 and out["gather_ok"] and out["gather_to_0_ok"]
    assert out["config"]["track_gather_ms"] is not None  # the FET track gather ran
    css = out["css"]
    assert set(css) == {"c3", "c4", "c5"}
    assert "track_gather_ms" in css["c4"] and "track_gather_ms" in css["c5"]
    assert css["c5"]["queue_each_once"] and sum(css["c5"]["chromosomes_per_rank"]) == 8
    # the ranks' stderr lines may interleave: count the notes, one per rank
    assert all(r.stderr.count(f"rank {k} reached the final barrier") == 1 for k in range(4)), r.stderr[-3000:]


def test_bench_single_rank_needs_no_launcher():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--dry-run"], capture_output=True, text=True,
                       timeout=120, cwd=ROOT)
    assert r.returncode == 0 and json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1
