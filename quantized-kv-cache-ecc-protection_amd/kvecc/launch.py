"""Self-launch of one process per GPU for bench.py and the Monte-Carlo sweep.

`python bench.py --gpus N` (or `tools/sweep.py --gpus N`) with no WORLD_SIZE
in the environment starts its N ranks itself, as child processes, BEFORE the
parent touches the GPU (the parent only counts devices, which does not
initialise HIP on this image, and never execs).  Each child gets the
torchrun-style environment (RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE,
MASTER_ADDR=127.0.0.1, MASTER_PORT) and re-runs the same script with the same
arguments; rank 0's stdout is the parent's stdout (the one JSON line), the
other ranks' stdout goes to stderr.  The parent exits non-zero when any rank
fails and stops the others.

Under torchrun (the driver's N > 1 form) WORLD_SIZE is already set and nothing
is spawned.  Counterpart of the process fan-out the reference does not have:
its sweep is one process on one GPU (evaluation/sweep.py:352-626); SURVEY §8(e)
asks for one process per GPU with a single RCCL all-reduce.
"""

from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time

ENV_LAUNCHED = "KVECC_LAUNCHED"


class LaunchError(RuntimeError):
    """The requested world cannot be formed on this machine."""


def free_port(host: str = "127.0.0.1") -> int:
    """An unused TCP port on `host` for the rendezvous."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def needs_spawn(gpus: int, environ=None) -> bool:
    """True when `gpus` ranks are asked for and no launcher has set the world up."""
    env = os.environ if environ is None else environ
    return gpus > 1 and "WORLD_SIZE" not in env and env.get(ENV_LAUNCHED) != "1"


def check_devices(gpus: int, backend: str, device_count: int) -> None:
    """Fail fast, before any rank starts, when the world cannot be formed:
    RCCL needs one GPU per rank; gloo may let ranks share the devices there are
    (to rehearse a multi-rank run on a one-GPU box) but needs at least one, and
    at most 16 ranks may use one GPU box at once."""
    if gpus < 1:
        raise LaunchError(f"--gpus must be >= 1, got {gpus}")
    if backend == "nccl" and device_count < gpus:
        raise LaunchError(f"--gpus {gpus} with the RCCL (nccl) backend needs {gpus} GPUs, "
                          f"this machine has {device_count}")
    if backend == "gloo":
        if device_count < 1:
            raise LaunchError(f"--gpus {gpus} --backend gloo needs at least one GPU, found none")
        if gpus > 16:
            raise LaunchError(f"--gpus {gpus}: at most 16 ranks may share the GPUs of one box")
    if backend not in ("nccl", "gloo"):
        raise LaunchError(f"unknown process-group backend {backend!r}")


def rank_env(rank: int, world: int, port: int, base=None) -> dict:
    """The torchrun-style environment of one child rank."""
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "GROUP_RANK": "0",
                "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), ENV_LAUNCHED: "1"})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts
    return env


def spawn(script, argv: list, world: int, timeout: float | None = None,
          poll: float = 0.2) -> int:
    """Run `python script *argv` as `world` ranks -- `script` a path, or the
    interpreter arguments that name the program, e.g. ["-m", "kvecc.montecarlo"]
    (the package root then joins each rank's PYTHONPATH) -- and return the launch's exit code:
    0 when every rank exited 0, else the first failing rank's code (a rank
    killed by a signal gives 128 + signal).  When one rank fails the others
    are terminated, so a rank stuck in a collective does not hang the launch."""
    port = free_port()
    prog = list(script) if isinstance(script, (list, tuple)) else [script]
    procs = []
    for r in range(world):
        out = None if r == 0 else 2  # fd 2: the other ranks' stdout joins stderr
        env = rank_env(r, world, port)
        if prog and prog[0] == "-m":  # a module: make its package importable in the rank
            root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
            env["PYTHONPATH"] = os.pathsep.join(p for p in (root, env.get("PYTHONPATH")) if p)
        procs.append(subprocess.Popen([sys.executable, *prog, *argv], env=env,
                                      stdout=out, start_new_session=True))
    t0 = time.monotonic()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                rc = c if c > 0 else 128 - c
                print(f"launch: rank {r} exited with {c}; stopping the other ranks", file=sys.stderr)
                break
            if all(c == 0 for c in codes):
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                print(f"launch: ranks still running after {timeout:.0f} s; stopping them", file=sys.stderr)
                rc = 124
                break
            time.sleep(poll)
    finally:
        _stop(procs)
    return rc


def _stop(procs, grace: float = 10.0) -> None:
    """Terminate every still-running rank (its own process group), then kill."""
    live = [p for p in procs if p.poll() is None]
    for p in live:
        try:
            os.killpg(p.pid, signal.SIGTERM)
        except (ProcessLookupError, PermissionError):
            pass
    t0 = time.monotonic()
    for p in live:
        try:
            p.wait(timeout=max(0.1, grace - (time.monotonic() - t0)))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            p.wait()


def launch_if_needed(script, argv: list, gpus: int, backend: str) -> int | None:
    """In the parent of a multi-rank run: check the devices, spawn the ranks and
    return the exit code for sys.exit.  In a rank (or a single-rank run): None."""
    if not needs_spawn(gpus):
        return None
    import torch  # device_count() does not initialise HIP on this image
    try:
        check_devices(gpus, backend, torch.cuda.device_count())
    except LaunchError as e:
        print(f"launch: {e}", file=sys.stderr)
        return 2
    return spawn(script, argv, gpus)


def check_world(dist, gpus: int) -> None:
    """In a rank: the process group must hold exactly the requested ranks."""
    got = dist.get_world_size()
    if got != gpus:
        raise LaunchError(f"--gpus {gpus} but the {dist.get_backend()} process group has "
                          f"{got} ranks")
