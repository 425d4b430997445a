"""Paged attention: the product (kvecc_paged_attention) against the matrix-core
kernels forced at G query heads per workgroup (tools/exp/attn_exp.hip,
libattnx.so), [B=8, ctx 4096, D=128], fp16 queries, random cache bytes (the
bench's worst case for the decode tables), MHA (32/32) and GQA (32q/8kv).
Times: mean per call over ITERS back-to-back calls bracketed by events, after
100 warm-up calls; outputs compared with the product's (max abs diff).

usage: python tools/exp/run_attn_exp.py [codec ...]
       python tools/exp/run_attn_exp.py packed_vec   (packed Golay MHA, 3 vs 4 codewords per lane)
"""
import ctypes
import math
import os
import sys

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
import torch  # noqa: E402

from kvecc import ops  # noqa: E402
from kvecc.memory_layout import kv_cache_pair  # noqa: E402

ITERS = int(os.environ.get("ITERS", "100"))
B, CTX, D, BS = 8, 4096, 128, 16
# (label, G, per_cu, fused)
VARIANTS = [("mfma_g1_cu4", 1, 4, 1), ("mfma_g1_cu2", 1, 2, 1), ("mfma_g1_cu8", 1, 8, 1),
            ("mfma_g1_cu4_nofuse", 1, 4, 0)]
GQA_VARIANTS = [("mfma_g4_cu4", 4, 4, 0), ("mfma_g4_cu4_fused", 4, 4, 1), ("mfma_g4_cu2_fused", 4, 2, 1),
                ("mfma_g4_cu8_fused", 4, 8, 1), ("mfma_g4_cu1", 4, 1, 0), ("mfma_g4_cu1_fused", 4, 1, 1)]


def main():
    dev = torch.device("cuda:0")
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "exp", "libattnx.so"))
    fn = lib.kvecc_exp_paged_attention_mfma
    vp, i64, ci, f32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_float
    fn.argtypes = [ci, ci, ci] + [vp] * 9 + [i64] * 9 + [f32, ci, vp, vp]
    codes = {"hamming84": 2, "golay": 3, "golay_packed": 4}
    pk = lib.kvecc_exp_paged_attention_packed
    pk.argtypes = [ci, ci] + [vp] * 8 + [i64] * 8 + [f32, vp, vp]
    if sys.argv[1:] == ["packed_vec"]:
        return packed_vec(dev, pk)
    if sys.argv[1:2] == ["gsp"]:
        gsp = lib.kvecc_exp_paged_attention_gsp
        gsp.argtypes = [ci, ci, ci, ci] + [vp] * 8 + [i64] * 8 + [f32, vp, vp]
        return golay_split_parity(dev, gsp, sys.argv[2:] or ["golay", "golay_packed"])
    for codec in (sys.argv[1:] or ["hamming84", "golay_packed", "golay"]):
        sets = ((32, 32, VARIANTS), (32, 8, GQA_VARIANTS))
        def parse_set(env):  # "label:G:per_cu:fused,..."
            return [(c.split(":")[0], *(int(x) for x in c.split(":")[1:])) for c in os.environ[env].split(",")]
        if os.environ.get("GQA_SET") or os.environ.get("MHA_SET"):  # only the sets given
            sets = tuple(x for x in ((32, 32, parse_set("MHA_SET") if os.environ.get("MHA_SET") else None),
                                     (32, 8, parse_set("GQA_SET") if os.environ.get("GQA_SET") else None))
                         if x[2])
        for heads, kvh, variants in sets:
            g = torch.Generator(device=dev).manual_seed(0)
            nb = CTX // BS
            blocks = B * nb
            per = D if codec == "hamming84" else (D + 2) // 3
            if codec == "golay_packed":
                per = (3 * per + 3) // 4 * 4
            kc, vc = kv_cache_pair((blocks, 1, kvh, BS * per), torch.int32 if codec == "golay" else torch.uint8, dev)
            kc.random_(0, 1 << 24 if codec == "golay" else 256, generator=g)
            vc.copy_(kc.roll(1, 0))
            ks = torch.rand(blocks, 1, kvh, BS, device=dev, generator=g)
            vs = torch.rand_like(ks)
            table = torch.randperm(blocks, device=dev, generator=g).to(torch.int32).view(B, nb)
            lens = torch.full((B,), CTX, dtype=torch.int32, device=dev)
            q = torch.randn(B, heads, D, device=dev, generator=g).half()
            ws = torch.empty(B * heads * 64 * (D + 2), dtype=torch.float32, device=dev)
            ref = torch.empty_like(q)
            out = torch.empty_like(q)
            s = torch.cuda.current_stream().cuda_stream
            sm = 1 / math.sqrt(D)

            def prod():
                ops.paged_attention_into(q, kc, vc, table, lens, ks, vs, ref, 0, BS, sm, codec, CTX)

            def var(G, per_cu, fused):
                def run():
                    rc = fn(G, per_cu, fused, q.data_ptr(), kc.data_ptr(), vc.data_ptr(), table.data_ptr(),
                            lens.data_ptr(), ks.data_ptr(), vs.data_ptr(), out.data_ptr(), B, heads, kvh, D,
                            blocks, 1, 0, BS, nb, CTX, sm, codes[codec], ws.data_ptr(), s)
                    assert rc == 0
                return run

            runs = [("product", prod)] + [(lab, var(G, pc, fu)) for lab, G, pc, fu in variants]
            res = {}
            for _ in range(2):  # two interleaved passes, the second reported
                for lab, run in runs:
                    for _ in range(100):
                        run()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(ITERS):
                        run()
                    e1.record()
                    torch.cuda.synchronize()
                    res[lab] = e0.elapsed_time(e1) * 1e3 / ITERS
            prod()
            torch.cuda.synchronize()
            for lab, run in runs:
                diff = 0.0
                if lab != "product":
                    run()
                    torch.cuda.synchronize()
                    diff = float((out.float() - ref.float()).abs().max())
                print(f"{codec:13s} {heads}q/{kvh}kv {lab:20s} {res[lab]:7.2f} us/call  maxdiff {diff:.3g}",
                      flush=True)
            del kc, vc, ws


def golay_split_parity(dev, gsp, codecs):
    """Golay MHA split kernel: spread parity table (sp 0, the product) vs two
    64-entry tables (sp 1), rows in flight (u, 0 = the product's), workgroups
    per CU of the split choice; random cache words; bit-equal outputs expected
    (same arithmetic)."""
    heads = kvh = 32
    for codec in codecs:
        packed = codec == "golay_packed"
        g = torch.Generator(device=dev).manual_seed(0)
        nb = CTX // BS
        blocks = B * nb
        per = (D + 2) // 3
        if packed:
            per = (3 * per + 3) // 4 * 4
        kc, vc = kv_cache_pair((blocks, 1, kvh, BS * per), torch.uint8 if packed else torch.int32, dev)
        kc.random_(0, 256 if packed else 1 << 24, generator=g)
        vc.copy_(kc.roll(1, 0))
        ks = torch.rand(blocks, 1, kvh, BS, device=dev, generator=g)
        vs = torch.rand_like(ks)
        table = torch.randperm(blocks, device=dev, generator=g).to(torch.int32).view(B, nb)
        lens = torch.full((B,), CTX, dtype=torch.int32, device=dev)
        q = torch.randn(B, heads, D, device=dev, generator=g).half()
        ws = torch.empty(B * heads * 64 * (D + 2), dtype=torch.float32, device=dev)
        ref = torch.empty_like(q)
        out = torch.empty_like(q)
        s = torch.cuda.current_stream().cuda_stream
        sm = 1 / math.sqrt(D)

        def prod():
            ops.paged_attention_into(q, kc, vc, table, lens, ks, vs, ref, 0, BS, sm, codec, CTX)

        def var(sp, u, per_cu):
            def run():
                rc = gsp(int(packed), sp, u, per_cu, q.data_ptr(), kc.data_ptr(), vc.data_ptr(), table.data_ptr(),
                         lens.data_ptr(), ks.data_ptr(), vs.data_ptr(), out.data_ptr(), B, heads, kvh, D, blocks, BS,
                         nb, CTX, sm, ws.data_ptr(), s)
                assert rc == 0, rc
            return run

        cfgs = os.environ.get("GSP_CFGS")  # "sp:u:cu,..." (sp 2: 6 codewords per lane, int32)
        if cfgs:
            cfgs = [tuple(int(x) for x in c.split(":")) for c in cfgs.split(",")]
        else:
            cfgs = ([(0, 0, 4), (1, 0, 4), (1, 0, 8), (1, 3, 4), (1, 3, 8), (1, 4, 4), (1, 4, 8), (0, 3, 4)]
                    if not packed else [(0, 0, 4), (1, 0, 4), (1, 0, 8), (1, 2, 8), (1, 3, 4), (1, 3, 8)])
        runs = [("product", prod)] + [(f"sp{a}_u{b}_cu{c}", var(a, b, c)) for a, b, c in cfgs]
        res = {lab: [] for lab, _ in runs}
        for _ in range(3):
            for lab, run in runs:
                for _ in range(100):
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(ITERS):
                    run()
                e1.record()
                torch.cuda.synchronize()
                res[lab].append(e0.elapsed_time(e1) * 1e3 / ITERS)
        prod()
        torch.cuda.synchronize()
        for lab, run in runs:
            diff = 0.0
            if lab != "product":
                run()
                torch.cuda.synchronize()
                diff = float((out.float() - ref.float()).abs().max())
            print(f"{codec:13s} {lab:16s} {min(res[lab]):7.2f} us/call (passes {', '.join(f'{x:.2f}' for x in res[lab])})"
                  f"  maxdiff {diff:.3g}", flush=True)
        del kc, vc, ws


def packed_vec(dev, pk):
    heads = kvh = 32
    g = torch.Generator(device=dev).manual_seed(0)
    nb = CTX // BS
    blocks = B * nb
    per = (3 * ((D + 2) // 3) + 3) // 4 * 4
    kc, vc = kv_cache_pair((blocks, 1, kvh, BS * per), torch.uint8, dev)
    kc.random_(0, 256, generator=g)
    vc.copy_(kc.roll(1, 0))
    ks = torch.rand(blocks, 1, kvh, BS, device=dev, generator=g)
    vs = torch.rand_like(ks)
    table = torch.randperm(blocks, device=dev, generator=g).to(torch.int32).view(B, nb)
    lens = torch.full((B,), CTX, dtype=torch.int32, device=dev)
    q = torch.randn(B, heads, D, device=dev, generator=g).half()
    ws = torch.empty(B * heads * 64 * (D + 2), dtype=torch.float32, device=dev)
    ref = torch.empty_like(q)
    out = torch.empty_like(q)
    s = torch.cuda.current_stream().cuda_stream
    sm = 1 / math.sqrt(D)

    def prod():
        ops.paged_attention_into(q, kc, vc, table, lens, ks, vs, ref, 0, BS, sm, "golay_packed", CTX)

    def var(vec, per_cu):
        def run():
            rc = pk(vec, per_cu, q.data_ptr(), kc.data_ptr(), vc.data_ptr(), table.data_ptr(), lens.data_ptr(),
                    ks.data_ptr(), vs.data_ptr(), out.data_ptr(), B, heads, kvh, D, blocks, BS, nb, CTX, sm,
                    ws.data_ptr(), s)
            assert rc == 0
        return run

    runs = [("product", prod), ("vec3_cu4", var(3, 4)), ("vec3_cu2", var(3, 2))]
    prev = os.environ.get("ATTN_PREV_LIB")  # the same kernels built from an earlier attention.hip
    if prev:
        pfn = ctypes.CDLL(os.path.abspath(prev)).kvecc_exp_paged_attention_packed
        pfn.argtypes = pk.argtypes

        def pvar(vec, per_cu):
            def run():
                rc = pfn(vec, per_cu, q.data_ptr(), kc.data_ptr(), vc.data_ptr(), table.data_ptr(), lens.data_ptr(),
                         ks.data_ptr(), vs.data_ptr(), out.data_ptr(), B, heads, kvh, D, blocks, BS, nb, CTX, sm,
                         ws.data_ptr(), s)
                assert rc == 0
            return run
        runs += [("prev_vec3_cu4", pvar(3, 4))]
    res = {}
    for _ in range(3):
        for lab, run in runs:
            for _ in range(50):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(ITERS):
                run()
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(lab, []).append(e0.elapsed_time(e1) * 1e3 / ITERS)
    prod()
    torch.cuda.synchronize()
    for lab, run in runs:
        diff = 0.0
        if lab != "product":
            run()
            torch.cuda.synchronize()
            diff = float((out.float() - ref.float()).abs().max())
        print(f"golay_packed  32q/32kv {lab:12s} {min(res[lab]):7.2f} us/call (passes {', '.join(f'{x:.1f}' for x in res[lab])})"
              f"  maxdiff {diff:.3g}", flush=True)


if __name__ == "__main__":
    main()
