"""A/B of the round-5 probes (tools/exp/r05_exp.hip) against the production
interpolation and decode+dequantize kernels at [8,4096,32,128], warm and back
to back as bench.py runs them: per variant, blocks of BLOCK launches between
two events, interleaved over ROUNDS rounds; median microseconds per launch.
Every variant's output (and statistics) is compared with production first.
usage (GPU box): python tools/exp/run_r05.py [interp|dd|all]   (env ROUNDS, BLOCK)"""
import ctypes
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch  # noqa: E402
from kvecc import ops  # noqa: E402

VP = ctypes.c_void_p
lib = ctypes.CDLL(os.path.join(HERE, "libr05.so"))
lib.r05_interp.argtypes = [ctypes.c_int, VP, VP, VP, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, VP]
lib.r05_interp_rec.argtypes = [ctypes.c_int, VP, VP, VP, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, VP,
                               ctypes.c_int32, VP]
lib.r05_dd.argtypes = [ctypes.c_int, VP, VP, VP, ctypes.c_int64, ctypes.c_int64, VP, VP]
lib.r05_quant.argtypes = [ctypes.c_int, VP, VP, VP, ctypes.c_int64, ctypes.c_int64, VP]
lib.r05_rows_enc.argtypes = [ctypes.c_int, VP, VP, ctypes.c_int64, ctypes.c_int64, VP]
lib.r05_pk_enc.argtypes = [ctypes.c_int, VP, VP, ctypes.c_int64, VP]
lib.r05_rows_dec.argtypes = [ctypes.c_int, VP, VP, ctypes.c_int64, ctypes.c_int64, VP, ctypes.c_int, VP]
lib.r05_dd32.argtypes = [ctypes.c_int, VP, VP, VP, ctypes.c_int64, ctypes.c_int64, VP, VP]
dev = torch.device("cuda:0")
S = VP(torch.cuda.current_stream().cuda_stream)
ROUNDS = int(os.environ.get("ROUNDS", "8"))
BLOCK = int(os.environ.get("BLOCK", "20"))
B, L, H, D = 8, 4096, 32, 128
P = lambda t: VP(t.data_ptr())  # noqa: E731
which = sys.argv[1] if len(sys.argv) > 1 else "all"


def ab(cases, nbytes, label):
    for fn in cases.values():  # warm-up
        for _ in range(30):
            fn()
    torch.cuda.synchronize()
    t = {k: [] for k in cases}
    for _ in range(ROUNDS):
        for k, fn in cases.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(BLOCK):
                fn()
            b.record()
            t[k].append((a, b))
    torch.cuda.synchronize()
    for k, v in sorted(t.items(), key=lambda kv: statistics.median(a.elapsed_time(b) for a, b in kv[1])):
        us = statistics.median(a.elapsed_time(b) * 1e3 / BLOCK for a, b in v)
        print(f"{label} {k:22s} {us:7.2f} us {nbytes / us / 1e3:6.0f} GB/s frac {nbytes / us / 8e6:5.3f}",
              flush=True)


if which in ("interp", "all"):
    g = torch.Generator().manual_seed(0)
    n = B * L * H * D
    x = torch.randint(0, 16, (n,), generator=g, dtype=torch.uint8).to(dev)
    cw = ops.hamming84_encode(x)
    ops.inject_into(cw, cw, 1e-3, 8, seed=42)
    q, et = torch.empty_like(x), torch.empty_like(x)
    ops.hamming84_decode_into(cw, q, et)
    del cw, x
    chunks = H * D // 16
    ref = torch.empty_like(q)
    ops.interpolate_into(q, et, ref, B, L, H * D)
    out = torch.empty_like(q)
    cases = {"prod": lambda: ops.interpolate_into(q, et, out, B, L, H * D)}
    for v in (0, 1, 2, 3, 4, 5, 10, 11, 12, 13, 14):
        cases[f"v{v}"] = (lambda v=v: lib.r05_interp(v, P(q), P(et), P(out), B, L, chunks, S))
    cases["api_auto"] = lambda: ops.interpolate_auto_into(q, et, out, B, L, H * D)
    flags = torch.zeros(2, dtype=torch.int32, device=dev)
    ep = [0]

    def rec(mode):
        ep[0] += 1
        return lib.r05_interp_rec(mode, P(q), P(et), P(out), B, L, chunks, P(flags), ep[0], S)
    for mode in range(3):
        cases[f"rec{mode}"] = (lambda mode=mode: rec(mode))
    for k, fn in cases.items():
        out.fill_(0xEE)
        rc = fn()
        torch.cuda.synchronize()
        print(f"interp {k}: rc={rc} equal={torch.equal(out, ref)}", flush=True)
    ab(cases, 3 * n, "interp")
    del q, et, ref, out

if which in ("dd", "all"):
    rows = B * L * H
    g = torch.Generator().manual_seed(1)
    cw = ops.hamming84_encode(torch.randint(0, 16, (rows * D,), generator=g, dtype=torch.uint8).to(dev))
    ops.inject_into(cw, cw, 1e-3, 8, seed=42)
    cw = cw.view(rows, D)
    sc = (torch.rand(rows, generator=g) * 0.1 + 0.01).to(dev)
    ref = torch.empty(rows, D, dtype=torch.float16, device=dev)
    st0 = ops.new_stats(dev)
    ops.decode_dequant_h84_into(cw, sc, ref, True, st0)
    out = torch.empty_like(ref)
    st = ops.new_stats(dev)
    cases = {"prod": lambda: ops.decode_dequant_h84_into(cw, sc, out, True, st)}
    for v in range(8):
        cases[f"v{v}"] = (lambda v=v: lib.r05_dd(v, P(cw), P(sc), P(out), rows, D, P(st), S))
    for k, fn in cases.items():
        out.fill_(float("nan"))
        st.zero_()
        rc = fn()
        torch.cuda.synchronize()
        print(f"dd {k}: rc={rc} equal={torch.equal(out, ref)} stats={ops.read_stats(st) == ops.read_stats(st0)}",
              flush=True)
    ab(cases, rows * (3 * D + 4), "dd_fp16")

if which in ("dd32", "all"):
    rows = B * L * H
    g = torch.Generator().manual_seed(1)
    cw = ops.hamming84_encode(torch.randint(0, 16, (rows * D,), generator=g, dtype=torch.uint8).to(dev))
    ops.inject_into(cw, cw, 1e-3, 8, seed=42)
    cw = cw.view(rows, D)
    sc = (torch.rand(rows, generator=g) * 0.1 + 0.01).to(dev)
    ref = torch.empty(rows, D, dtype=torch.float32, device=dev)
    st0 = ops.new_stats(dev)
    ops.decode_dequant_h84_into(cw, sc, ref, True, st0)
    out = torch.empty_like(ref)
    st = ops.new_stats(dev)
    cases = {"prod": lambda: ops.decode_dequant_h84_into(cw, sc, out, True, st)}
    for v in range(5):
        cases[f"v{v}"] = (lambda v=v: lib.r05_dd32(v, P(cw), P(sc), P(out), rows, D, P(st), S))
    for k, fn in cases.items():
        out.fill_(float("nan"))
        st.zero_()
        rc = fn()
        torch.cuda.synchronize()
        print(f"dd32 {k}: rc={rc if isinstance(rc, int) else 0} equal={torch.equal(out, ref)} "
              f"stats={ops.read_stats(st) == ops.read_stats(st0)}", flush=True)
    ab(cases, rows * (5 * D + 4), "dd_fp32")

if which in ("quant", "all"):
    from kvecc import _lib
    rows = B * L * H
    g = torch.Generator().manual_seed(5)
    x = torch.randn(rows, D, generator=g).to(dev).to(torch.float16)
    cw0 = torch.empty(rows, D, dtype=torch.uint8, device=dev)
    sc0 = torch.empty(rows, dtype=torch.float32, device=dev)
    ops.quantize_encode_rows_into(x, _lib.CODEC_H84, cw0, sc0)
    cw = torch.empty_like(cw0)
    sc = torch.empty_like(sc0)
    cases = {"prod": lambda: ops.quantize_encode_rows_into(x, _lib.CODEC_H84, cw, sc)}
    for v in range(4):
        cases[f"v{v}"] = (lambda v=v: lib.r05_quant(v, P(x), P(cw), P(sc), rows, D, S))
    for k, fn in cases.items():
        cw.zero_()
        sc.zero_()
        fn()
        torch.cuda.synchronize()
        print(f"quant {k}: equal={torch.equal(cw, cw0) and torch.equal(sc, sc0)}", flush=True)
    ab(cases, rows * (3 * D + 4), "quant_fp16")

if which in ("rows", "all"):
    rows = B * L * H
    g = torch.Generator().manual_seed(9)
    x = torch.randint(0, 16, (rows, D), generator=g, dtype=torch.uint8).to(dev)
    G = (D + 2) // 3
    ref = torch.empty(rows, G, dtype=torch.int32, device=dev)
    ops.golay_encode_rows_into(x, ref)
    out = torch.empty_like(ref)
    cases = {"prod": lambda: ops.golay_encode_rows_into(x, out)}
    for v in (0, 8, 9):
        cases[f"v{v}"] = (lambda v=v: lib.r05_rows_enc(v, P(x), P(out), rows, D, S))
    for k, fn in cases.items():
        out.zero_()
        rc = fn()
        torch.cuda.synchronize()
        print(f"rows_enc {k}: rc={rc} equal={torch.equal(out, ref)}", flush=True)
    ab(cases, rows * (D + 4 * G), "rows_enc")

if which in ("pk", "all"):
    m = 45088768  # the headline's per-head codewords (bench.py packed section)
    g = torch.Generator().manual_seed(11)
    nib = torch.randint(0, 256, (m * 3 // 2,), generator=g, dtype=torch.uint8).to(dev)
    ref = ops.golay_encode_packed(nib, m)
    out = torch.empty_like(ref)
    cases = {"prod": lambda: ops.golay_encode_packed_into(nib, out, m)}
    for v in range(5):
        cases[f"v{v}"] = (lambda v=v: lib.r05_pk_enc(v, P(nib), P(out), m, S))
    for k, fn in cases.items():
        out.zero_()
        rc = fn()
        torch.cuda.synchronize()
        print(f"pk_enc {k}: rc={rc} equal={torch.equal(out, ref)}", flush=True)
    ab(cases, int(4.5 * m), "pk_enc")

if which in ("rowsdec", "all"):
    rows = B * L * H
    G = (D + 2) // 3
    g = torch.Generator().manual_seed(13)
    x = torch.randint(0, 16, (rows, D), generator=g, dtype=torch.uint8).to(dev)
    cw = ops.golay_encode_rows(x).view(-1)
    ops.inject_into(cw, cw, 1e-2, 24, seed=42)
    cw = cw.view(rows, G)
    ref = torch.empty(rows, D, dtype=torch.uint8, device=dev)
    st0 = ops.new_stats(dev)
    ops.golay_decode_rows_into(cw, ref, stats=st0)
    out = torch.empty_like(ref)
    st = ops.new_stats(dev)
    cases = {"prod": lambda: ops.golay_decode_rows_into(cw, out, stats=st)}
    for v, pc in ((0, 2), (1, 2), (2, 2), (3, 3), (4, 3), (5, 3), (6, 3), (5, 4), (3, 4)):
        cases[f"v{v}:{pc}"] = (lambda v=v, pc=pc: lib.r05_rows_dec(v, P(cw), P(out), rows, D, P(st), pc, S))
    for k, fn in cases.items():
        out.zero_()
        st.zero_()
        rc = fn()
        torch.cuda.synchronize()
        print(f"rows_dec {k}: rc={rc} equal={torch.equal(out, ref)} stats={ops.read_stats(st) == ops.read_stats(st0)}",
              flush=True)
    ab(cases, rows * (4 * G + D), "rows_dec")
