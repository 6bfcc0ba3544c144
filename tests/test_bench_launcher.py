"""bench.py's own rank launcher (no GPU): ``--gpus N`` with WORLD_SIZE unset starts N rank
processes with the torch.distributed environment (before any GPU work) and rank 0 reports the
world size; a torch.distributed.run launch must agree with ``--gpus``."""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def test_launcher_spawns_ranks():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout          # rank 0 only
    out = json.loads(lines[0])
    assert out["dry_run"] and out["n_gpus"] == 2 and out["ranks"] == 2
    # the N-GPU line's self-diagnosis (rank_diagnostics): gathered from every rank over gloo
    diag = out["rank_diagnostics"]
    for k in ("ranks", "rccl_nranks", "kernel_ms_max", "kernel_ms_min", "kernel_skew",
              "allgather_us_per_call_max", "per_rank"):
        assert k in diag, k
    assert diag["ranks"] == 2 and len(diag["per_rank"]) == 2
    assert all(set(r) == {"kernel_ms", "allgather_us"} for r in diag["per_rank"])


def test_world_size_must_match_gpus():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"],
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    assert "WORLD_SIZE=1" in (p.stderr + p.stdout)
