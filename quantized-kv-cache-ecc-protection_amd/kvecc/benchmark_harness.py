"""Codec micro-benchmarks with the API of kv_cache/benchmark_harness.py
(BenchmarkResult :18-26, cuda_timer :42-57, benchmark_* :60-210), timing the
HIP backend.  Same semantics: inputs resident on the GPU, `repeat` launches
between two events after `warmup` launches, latency in us per call (including
the Python-int stats sync the reference-compatible wrappers perform), and
throughput in values per us (= M values/s)."""

from __future__ import annotations

from dataclasses import dataclass

import torch

from . import ops


@dataclass
class BenchmarkResult:
    name: str
    n_elements: int
    n_bits: int
    latency_us: float
    throughput_mvals_sec: float
    extra: dict | None = None


def cuda_timer(func, warmup=10, repeat=100):
    for _ in range(warmup):
        func()
    torch.cuda.synchronize()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record()
    for _ in range(repeat):
        func()
    end.record()
    torch.cuda.synchronize()
    return start.elapsed_time(end) * 1000 / repeat


def _result(name, n, n_bits, us, extra=None):
    return BenchmarkResult(name=name, n_elements=n, n_bits=n_bits, latency_us=us,
                           throughput_mvals_sec=n / us, extra=extra)


def benchmark_hamming84_encode(n_elements=1_000_000, warmup=10, repeat=100):
    data = torch.randint(0, 16, (n_elements,), dtype=torch.uint8, device="cuda")
    return _result("hamming84_encode", n_elements, 8,
                   cuda_timer(lambda: ops.hamming84_encode(data), warmup, repeat))


def benchmark_hamming84_decode(n_elements=1_000_000, warmup=10, repeat=100):
    enc = ops.hamming84_encode(torch.randint(0, 16, (n_elements,), dtype=torch.uint8, device="cuda"))
    return _result("hamming84_decode", n_elements, 8,
                   cuda_timer(lambda: ops.hamming84_decode(enc), warmup, repeat))


def benchmark_golay_encode(n_triplets=333_333, warmup=10, repeat=100):
    trip = torch.randint(0, 16, (n_triplets, 3), dtype=torch.uint8, device="cuda")
    return _result("golay_encode", n_triplets * 3, 24,
                   cuda_timer(lambda: ops.golay_encode(trip), warmup, repeat))


def benchmark_golay_decode(n_triplets=333_333, warmup=10, repeat=100):
    enc = ops.golay_encode(torch.randint(0, 16, (n_triplets, 3), dtype=torch.uint8, device="cuda"))
    return _result("golay_decode", n_triplets * 3, 24,
                   cuda_timer(lambda: ops.golay_decode(enc), warmup, repeat))


def benchmark_fault_injection(n_elements=1_000_000, ber=0.01, n_bits=8, warmup=10, repeat=100):
    if n_bits <= 8:
        data = torch.randint(0, 256, (n_elements,), dtype=torch.uint8, device="cuda")
    else:
        data = torch.randint(0, 2 ** 24, (n_elements,), dtype=torch.int32, device="cuda")
    us = cuda_timer(lambda: ops.inject_bit_errors_triton(data, ber, n_bits, 42), warmup, repeat)
    return _result(f"fault_injection_ber{ber}", n_elements, n_bits, us, {"ber": ber})


def benchmark_encode_inject_decode(codec="hamming84", n_elements=1_000_000, ber=0.01, warmup=10,
                                   repeat=100):
    if codec == "hamming84":
        data = torch.randint(0, 16, (n_elements,), dtype=torch.uint8, device="cuda")
        n_bits = 8

        def pipeline():
            enc = ops.hamming84_encode(data)
            return ops.hamming84_decode(ops.inject_bit_errors_triton(enc, ber, n_bits, seed=42))[0]
    else:
        trip = torch.randint(0, 16, ((n_elements + 2) // 3, 3), dtype=torch.uint8, device="cuda")
        n_bits = 24

        def pipeline():
            enc = ops.golay_encode(trip)
            return ops.golay_decode(ops.inject_bit_errors_triton(enc, ber, n_bits, seed=42))[0]
    us = cuda_timer(pipeline, warmup, repeat)
    return _result(f"{codec}_pipeline_ber{ber}", n_elements, n_bits, us, {"codec": codec, "ber": ber})
