"""The self-launcher of bench.py / tools/sweep.py (kvecc.launch): argument and
environment plumbing, fail-fast checks, and a real gloo rendezvous of spawned
ranks on the CPU.  The HIP form (`bench.py --gpus 2 --backend gloo` on one GPU)
is tests/test_gpu_launch.py."""

import json
import os
import subprocess
import sys
import textwrap

import pytest

from kvecc import launch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_needs_spawn():
    assert not launch.needs_spawn(1, {})
    assert launch.needs_spawn(2, {})
    assert not launch.needs_spawn(2, {"WORLD_SIZE": "2"})          # torchrun set the world up
    assert not launch.needs_spawn(8, {launch.ENV_LAUNCHED: "1"})    # a spawned rank


def test_check_devices():
    launch.check_devices(1, "nccl", 1)
    launch.check_devices(8, "nccl", 8)
    launch.check_devices(2, "gloo", 1)      # ranks share the one GPU
    with pytest.raises(launch.LaunchError, match="needs 8 GPUs"):
        launch.check_devices(8, "nccl", 1)
    with pytest.raises(launch.LaunchError, match="at least one GPU"):
        launch.check_devices(2, "gloo", 0)
    with pytest.raises(launch.LaunchError, match="at most 16"):
        launch.check_devices(17, "gloo", 1)
    with pytest.raises(launch.LaunchError):
        launch.check_devices(0, "nccl", 8)
    with pytest.raises(launch.LaunchError, match="backend"):
        launch.check_devices(2, "mpi", 8)


def test_rank_env():
    env = launch.rank_env(3, 4, 29999, base={"PATH": "/bin"})
    assert env["RANK"] == env["LOCAL_RANK"] == "3"
    assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "4"
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29999"
    assert env[launch.ENV_LAUNCHED] == "1" and env["PATH"] == "/bin"
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


_RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys, torch, torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([int(os.environ["RANK"]) + 1], dtype=torch.int64)
    dist.all_reduce(t)
    fail = int(sys.argv[1]) if len(sys.argv) > 1 else -1
    if dist.get_rank() == fail:
        sys.exit(7)
    if dist.get_rank() == 0:
        print(json.dumps({"world": dist.get_world_size(), "sum": int(t), "argv": sys.argv[1:]}))
    dist.destroy_process_group()
""")


def _run_launcher(tmp_path, world, *argv, timeout=None):
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    code = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd")!r})
        from kvecc import launch
        sys.exit(launch.spawn({str(script)!r}, {list(argv)!r}, {world}, timeout={timeout!r}))
    """)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", launch.ENV_LAUNCHED)}
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)


def test_spawn_gloo_world(tmp_path):
    """Spawned ranks rendezvous over 127.0.0.1; only rank 0's stdout reaches stdout."""
    r = _run_launcher(tmp_path, 3, "-1")
    assert r.returncode == 0, r.stderr
    # gloo itself prints a "[Gloo] Rank 0 is connected" line on rank 0's stdout
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    assert json.loads(lines[0]) == {"world": 3, "sum": 6, "argv": ["-1"]}


def test_spawn_failing_rank_fails_launch(tmp_path):
    """One rank exits 7: the launch exits 7 and stops the others."""
    r = _run_launcher(tmp_path, 2, "1")
    assert r.returncode == 7, (r.returncode, r.stderr)
    assert "rank 1 exited with 7" in r.stderr


def test_bench_fails_fast_without_enough_gpus():
    """`bench.py --gpus 8` where 8 GPUs do not exist exits non-zero before any rank starts."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", launch.ENV_LAUNCHED)}
    env["HIP_VISIBLE_DEVICES"] = ""  # no devices, whatever the machine has
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2, r.stderr
    assert "needs 8 GPUs" in r.stderr and r.stdout.strip() == ""


def test_bench_rejects_mismatched_world():
    """A launcher's WORLD_SIZE that disagrees with --gpus is an error, not a warning."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2, r.stderr
    assert "WORLD_SIZE=1" in r.stderr


def test_sweep_fails_fast_without_enough_gpus():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", launch.ENV_LAUNCHED)}
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "sweep.py"), "--gpus", "4"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2, r.stderr
    assert "needs 4 GPUs" in r.stderr


def test_bench_strong_scaling_rejects_more_ranks_than_rows():
    """--scaling strong splits the B=8 rows of the one tensor: 9 ranks is an error before any GPU work."""
    env = dict(os.environ, WORLD_SIZE="9", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "9", "--scaling", "strong",
                        "--steps", "1"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 2, r.stderr
    assert "at most 8 ranks" in r.stderr


def test_bench_sections_flag():
    """--sections keeps exactly the named sections; an unknown name is a usage error."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    a = bench.parse(["--sections", "montecarlo,strong"])
    assert not a.no_montecarlo and not a.no_strong
    assert all(getattr(a, f) for s, f in bench.SECTIONS.items() if s not in ("montecarlo", "strong"))
    a = bench.parse(["--no-sections"])
    assert all(getattr(a, f) for f in bench.SECTIONS.values())
    a = bench.parse([])
    assert a.gpus is None and not any(getattr(a, f) for f in bench.SECTIONS.values())
    with pytest.raises(SystemExit):
        bench.parse(["--sections", "nope"])


def test_spawn_module_form(tmp_path):
    """spawn(["-m", module]) runs a module entry point in every rank (the sweep's
    self-launch: `python -m kvecc.montecarlo --gpus N`), with kvecc importable."""
    pkg = tmp_path / "mod_pkg"
    pkg.mkdir()
    (pkg / "__init__.py").write_text("")
    (pkg / "rank.py").write_text("import kvecc.launch\n" + _RANK_SCRIPT)
    code = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd")!r})
        from kvecc import launch
        sys.exit(launch.spawn(["-m", "mod_pkg.rank"], ["-1"], 2))
    """)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", launch.ENV_LAUNCHED)}
    env.pop("PYTHONPATH", None)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env,
                       cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert json.loads(lines[0]) == {"world": 2, "sum": 3, "argv": ["-1"]}
