"""Historical (round 3): needs a -DKVECC_SHIM_WAVE_TIMES=1 build of csrc/shim.hip; round 4
removed the switch (results in profiles/r03/fused/wave_times_*.log).

Per-wave start / exit times of the fused Golay read (a build with
-DKVECC_SHIM_WAVE_TIMES=1): how evenly the persistent grid's waves finish.
usage: python tools/exp/run_wave_times.py libread_times.so"""
import ctypes, os, sys
REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "quantized-kv-cache-ecc-protection_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402
from kvecc import _lib, ops  # noqa: E402
import run_read_ab as ab  # noqa: E402

dev = torch.device("cuda:0")
h = ctypes.CDLL(os.path.abspath(sys.argv[1]))
fn = h.kvecc_shim_read_batch
fn.argtypes = _lib.SIGNATURES["kvecc_shim_read_batch"]
h.kvecc_exp_wave_times.argtypes = [ctypes.c_void_p]
B, L, H, D, BS = ab.B, ab.L, ab.H, ab.D, ab.BS
nb = B * (L // BS)
gen = torch.Generator().manual_seed(7)
table = torch.randperm(nb, generator=gen).to(torch.int32).view(B, L // BS).to(dev)
scales = [(torch.rand(nb, 1, H, BS, generator=gen) * 0.1 + 0.01).to(dev) for _ in range(2)]
for packed in (False, True):
    caches = ab.golay_caches(dev, packed, gen, nb)
    g = (D + 2) // 3
    per = ((3 * g + 3) // 4 * 4) if packed else g
    bs = caches[0].shape[-1] // per
    outs = [torch.empty(B, H, L, D, dtype=torch.float16, device=dev) for _ in range(2)]
    st = ops.new_stats(dev)
    times = torch.zeros(3 * 65536, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for rep in range(4):
        times.zero_()
        torch.cuda.synchronize()
        assert h.kvecc_exp_wave_times(ctypes.c_void_p(times.data_ptr())) == 0
        rc = fn(caches[0].data_ptr(), caches[1].data_ptr(), scales[0].data_ptr(), scales[1].data_ptr(),
                table.data_ptr(), table.shape[1], B, L, H, D, 1, bs, 0, 4 if packed else 3, 0,
                outs[0].data_ptr(), outs[1].data_ptr(), ops._DT[torch.float16], st.data_ptr(), stream)
        assert rc == 0
        torch.cuda.synchronize()
    t = times.view(-1, 3).cpu()
    t = t[t[:, 1] > 0]
    if len(sys.argv) > 2:
        import numpy as np
        np.save(f"{sys.argv[2]}_{'packed' if packed else 'int32'}.npy", t.numpy())
    t0 = int(t[:, 0].min())
    st_ = (t[:, 0] - t0).double() / 100.0  # 100 MHz -> us
    en = (t[:, 1] - t0).double() / 100.0
    q = torch.tensor([0.0, 0.01, 0.1, 0.5, 0.9, 0.99, 1.0], dtype=torch.float64)
    print(f"{'packed' if packed else 'int32'}: {t.shape[0]} waves; start quantiles (us) "
          f"{[round(float(x), 1) for x in torch.quantile(st_, q)]}")
    print(f"   end quantiles (us) {[round(float(x), 1) for x in torch.quantile(en, q)]}")
    # finish times by XCD (dispatch deals workgroups round-robin over 8 XCDs)
    nt = t[:, 2].double()
    print(f"   tiles per wave: min {int(nt.min())} median {float(nt.median()):.0f} max {int(nt.max())}; "
          f"corr(tiles, end) {float(torch.corrcoef(torch.stack([nt, en]))[0, 1]):.2f}")
    fast = en < torch.quantile(en, 0.1)
    slow = en > torch.quantile(en, 0.9)
    print(f"   tiles: fastest 10% of waves {float(nt[fast].mean()):.1f}, slowest 10% {float(nt[slow].mean()):.1f}")
    wg = torch.arange(t.shape[0]) // 8
    for x in range(8):
        sel = en[(wg % 8) == x]
        print(f"   xcd {x}: median end {float(sel.median()):.1f} us, max {float(sel.max()):.1f}")
