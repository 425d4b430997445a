"""Issue cost of single VALU instructions on gfx950 (tools/exp/valu_rate.hip):
cycles per wave-instruction per SIMD with every SIMD full, at the 2.4 GHz clock.
usage (GPU box): python tools/exp/run_valu_rate.py"""
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libvalu.so"))
lib.valu_rate.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
NAMES = ["v_add_u32", "v_xor_b32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_u32_u24", "v_add_f32", "v_fma_f32",
         "v_bitop3_b32(xor3)", "v_add3_u32", "v_lshlrev_b32", "v_mul_hi_u32_u24", "v_mad_u32_u24"]
CUS, SIMDS, CLK = 256, 4, 2.4e9
blocks = CUS * 8 * 4  # 8 waves per SIMD, 4 rounds of residency
iters = 2000
out = torch.empty(blocks * 256, dtype=torch.int32, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
res = {}
for op, name in enumerate(NAMES):
    for _ in range(3):
        assert lib.valu_rate(op, ctypes.c_void_p(out.data_ptr()), blocks, iters, s) == 0
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        lib.valu_rate(op, ctypes.c_void_p(out.data_ptr()), blocks, iters, s)
    b.record()
    torch.cuda.synchronize()
    sec = a.elapsed_time(b) / 5 * 1e-3
    waves = blocks * 4
    instrs = waves * 8 * iters
    cyc = sec * CLK * CUS * SIMDS / instrs
    res[name] = {"us": sec * 1e6, "cycles_per_wave_instr_per_simd": cyc,
                 "wave_instr_per_s": instrs / sec}
    print(f"{name:18s} {sec * 1e6:9.1f} us  {cyc:5.2f} cycles/wave-instr/SIMD  {instrs / sec:.3e} wave-instr/s",
          flush=True)
print(json.dumps(res))
