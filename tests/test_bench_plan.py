"""bench.py's multi-GPU launch on CPU: `--gpus 2` spawns two worker processes itself (the parent
never touches the GPU), they rendezvous over gloo on 127.0.0.1 and batch-shard SURVEY config 3
(1 024 × 256 residues, LPT) — `--plan` stops before any GPU work."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _plan(*flags):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--plan", *flags], capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


@pytest.mark.parametrize("n", [2, 4])
def test_bench_spawns_and_shards_config3(n):
    p = _plan("--gpus", str(n))
    assert p["n_gpus"] == n and p["world_size_seen"] == n
    assert p["residues_job"] == 262144 and p["proteins_job"] == 1024
    assert p["proteins_per_rank"] == [1024 // n] * n and p["disjoint"]
    assert p["scaling"] == "strong"


def test_bench_weak_mode_plan():
    p = _plan("--gpus", "2", "--weak")
    assert p["residues_job"] == 2 * 262144 and p["proteins_per_rank"] == [1024, 1024] and p["disjoint"]


def test_bench_defines_every_leg():
    """Every function bench.py's main() calls on the GPU box exists (a CPU run only exercises
    --plan): the timed loop's helpers and each reported leg."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    for name in ("workload", "reference_exact_match", "clock_stats", "casp14_end_to_end", "cpu_baselines",
                 "_ref_as_computed_rate", "spawn_workers", "plan_only", "host_cores", "init_group", "shard_ids"):
        assert callable(getattr(m, name, None)), name
    src = open(spec.origin).read()
    import ast
    called = {n.func.id for n in ast.walk(ast.parse(src)) if isinstance(n, ast.Call) and isinstance(n.func, ast.Name)}
    tree = ast.parse(src)
    defined = {n.name for n in ast.walk(tree) if isinstance(n, ast.FunctionDef)}
    defined |= {a.asname or a.name for n in ast.walk(tree) if isinstance(n, (ast.Import, ast.ImportFrom)) for a in n.names}
    import builtins
    missing = {c for c in called if c not in defined and not hasattr(builtins, c)} - {"O", "P"}
    assert not missing, missing
