"""bench.py / tools/sweep.py start their own ranks on a GPU box (kvecc.launch).

On a one-GPU box two ranks share cuda:0 over gloo (RCCL refuses two ranks on
one device); the JSON line must report the world the process group itself
reports.  Asking for more GPUs than the box has fails before any rank starts.
"""

import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    from kvecc import launch
    return {k: v for k, v in os.environ.items()
            if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", launch.ENV_LAUNCHED)}


def _json_line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_spawns_two_gloo_ranks(gpu):
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--steps", "10", "--warmup", "2", "--no-cpu-baseline", "--no-inject", "--no-packed",
                        "--no-fused", "--no-rows", "--roofline-samples", "2", "--no-sections"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 2
    assert line["config"]["process_group"] == {"backend": "gloo", "world_size": 2}
    assert line["config"]["launcher"].startswith("self")
    ranks = line["config"]["per_rank"]
    assert [p["rank"] for p in ranks] == [0, 1]
    assert all(p["decode_ms"] > 0 and p["encode_ms"] > 0 for p in ranks)
    # value = every rank's codewords over the slowest rank's time
    m = line["config"]["codewords_per_gpu"]
    slowest = max(p["elapsed_s"] for p in ranks)
    assert line["value"] == pytest.approx(2 * m * line["steps"] / slowest, rel=1e-6)
    # the decode statistics are the all-reduced sum of both shards
    assert line["decode_stats"]["bits_corrected"] > 0


@pytest.mark.gpu
def test_bench_rccl_world1(gpu):
    """The RCCL path of the multi-GPU bench (init with device_id, barriers, the
    per-rank all_gather and the statistics all_reduce) on a real "nccl" group of
    one rank -- what every rank of the driver's 8-GPU run executes."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--dist",
                        "--steps", "10", "--warmup", "2", "--no-cpu-baseline", "--no-inject", "--no-packed",
                        "--no-fused", "--no-rows", "--roofline-samples", "2", "--no-sections"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 1
    assert line["config"]["process_group"] == {"backend": "nccl", "world_size": 1}
    assert [p["rank"] for p in line["config"]["per_rank"]] == [0]
    assert line["decode_stats"]["bits_corrected"] > 0


@pytest.mark.gpu
def test_bench_more_gpus_than_the_box_fails(gpu):
    import torch
    n = torch.cuda.device_count() + 1
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env=_env())
    assert r.returncode != 0
    assert f"needs {n} GPUs" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.gpu
def test_sweep_spawns_two_gloo_ranks_equal_to_one(gpu, tmp_path):
    """tools/sweep.py --gpus 2 (spawned, gloo, sharing cuda:0) gives the single-rank table."""
    args = ["--shape", "4", "64", "4", "32", "--codecs", "hamming84_interp", "golay",
            "--bers", "1e-2", "--seeds", "42"]
    one = subprocess.run([sys.executable, os.path.join(REPO, "tools", "sweep.py"), *args],
                         capture_output=True, text=True, timeout=180, env=_env())
    assert one.returncode == 0, one.stderr[-3000:]
    two = subprocess.run([sys.executable, os.path.join(REPO, "tools", "sweep.py"), "--gpus", "2",
                          "--backend", "gloo", *args], capture_output=True, text=True, timeout=180, env=_env())
    assert two.returncode == 0, two.stderr[-3000:]

    def rows(out):
        rs = [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]
        return [r for r in rs if "key" in r], rs[-1]

    r1, s1 = rows(one.stdout)
    r2, s2 = rows(two.stdout)
    assert s1["world"] == 1 and s2["world"] == 2 and s2["backend"] == "gloo"
    assert r1 == r2 and len(r1) == 2


def _bench(*args, timeout=300):
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args],
                       capture_output=True, text=True, timeout=timeout, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    return _json_line(r.stdout)


@pytest.mark.gpu
def test_bench_sharded_sweep_and_strong_scaling_equal_one_rank(gpu):
    """What the driver's N-GPU run records beside the weak headline: the config-5
    sweep batch-sharded over the ranks with its one all-reduce, and the strong-
    scaling split of the headline tensor.  Two gloo ranks sharing cuda:0 must
    give the single rank's counter table (same sha256) and the same all-reduced
    decode / injection statistics."""
    common = ["--steps", "3", "--warmup", "1", "--roofline-samples", "1", "--sections", "montecarlo,strong"]
    one = _bench("--gpus", "1", *common)
    two = _bench("--gpus", "2", "--backend", "gloo", *common)
    m1, m2 = one["montecarlo"], two["montecarlo"]
    assert m1["world"] == 1 and m2["world"] == 2 and m1["trials"] == m2["trials"] == 36
    assert m2["table_sha256"] == m1["table_sha256"]
    assert [p["batch_rows"] for p in m2["per_rank"]] == [[0, 4], [4, 8]]
    assert m2["collective"].endswith("(gloo)") and m1["collective"] is None
    assert m2["ms"] == pytest.approx(max(p["ms"] for p in m2["per_rank"]))
    s1, s2 = one["strong_scaling"], two["strong_scaling"]
    assert s1["world"] == 1 and s2["world"] == 2
    assert s1["codewords_total"] == s2["codewords_total"] == 8 * 4096 * 32 * 43
    assert sum(p["codewords"] for p in s2["per_rank"]) == s2["codewords_total"]
    assert s2["decode_stats"] == s1["decode_stats"] and s2["inject_stats"] == s1["inject_stats"]
    assert s1["decode_stats"]["bits_corrected"] > 0


@pytest.mark.gpu
def test_bench_strong_headline_two_ranks(gpu):
    """--scaling strong: the headline itself splits the one tensor; value counts
    the whole tensor per step over the slowest rank, statistics equal one rank's."""
    common = ["--steps", "4", "--warmup", "1", "--roofline-samples", "1", "--no-sections", "--scaling", "strong"]
    one = _bench("--gpus", "1", *common)
    two = _bench("--gpus", "2", "--backend", "gloo", *common)
    assert one["scaling"] == two["scaling"] == "strong"
    total = 8 * 4096 * 32 * 43
    assert two["config"]["codewords_per_step"] == total and two["config"]["codewords_per_gpu"] == total // 2
    slowest = max(p["elapsed_s"] for p in two["config"]["per_rank"])
    assert two["value"] == pytest.approx(total * 4 / slowest, rel=1e-6)
    assert two["decode_stats"] == one["decode_stats"]


@pytest.mark.gpu
def test_bench_under_torchrun_takes_the_launchers_world(gpu):
    """The driver's form: torchrun starts the ranks; --gpus may be omitted (it
    then comes from WORLD_SIZE) and nothing is spawned a second time."""
    from kvecc import launch
    port = launch.free_port()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"),
                        "--backend", "gloo", "--steps", "3", "--warmup", "1", "--roofline-samples", "1",
                        "--sections", "montecarlo"],
                       capture_output=True, text=True, timeout=300, env=_env())
    assert r.returncode == 0, r.stderr[-3000:]
    line = _json_line(r.stdout)
    assert line["n_gpus"] == 2 and line["config"]["launcher"] == "external (torchrun)"
    assert line["config"]["process_group"] == {"backend": "gloo", "world_size": 2}
    assert line["montecarlo"]["world"] == 2 and len(line["montecarlo"]["per_rank"]) == 2
