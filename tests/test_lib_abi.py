"""CPU-only checks of the C ABI library (no kernel launches).

* libkvecc.so loads and exports every function include/kvecc.h declares;
* the host-side code tables of the product equal the oracle's (and hence the
  reference's golden table);
* the integer BER threshold the kernels use is exactly the reference's
  fp32 `tl.rand < ber` test.
"""

import ctypes
import os
import re

import numpy as np
import pytest

from tests.conftest import REPO

HEADER = os.path.join(REPO, "include", "kvecc.h")


def _declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"KVECC_API\s+[\w\s\*]+?\b(kvecc_\w+)\s*\(", text)))


def test_header_declares_api():
    names = _declared()
    assert "kvecc_golay_decode" in names and "kvecc_inject_u8" in names
    assert len(names) >= 25


def test_library_exports_every_declared_symbol():
    from kvecc import _lib
    lib = _lib.load()
    for name in _declared():
        assert hasattr(lib, name), name
    # and the Python binding covers the whole ABI
    assert set(_declared()) == set(_lib.SIGNATURES)


def test_exported_symbols_are_only_the_abi():
    """-fvisibility=hidden: nothing but kvecc_* leaks from the library."""
    import subprocess
    from kvecc import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert syms and all(s.startswith("kvecc_") for s in syms), sorted(syms)[:10]


def test_version_and_no_device_errors():
    from kvecc import _lib
    assert _lib.version().startswith("kvecc")
    lib = _lib.load()
    # argument validation runs before any device work
    rc = lib.kvecc_hamming84_encode(None, None, -1, None)
    assert rc == -1 and b"negative" in lib.kvecc_last_error()
    assert lib.kvecc_hamming84_encode(None, None, 0, None) == 0  # empty is valid


def test_golay_tables_match_oracle(oracle, golden):
    from kvecc import config
    t = config.build_golay_syndrome_table().numpy()
    assert np.array_equal(t, oracle.golay_syndrome_table())
    assert np.array_equal(t, golden("golay")["table"])
    masks = np.zeros(12, np.uint32)
    from kvecc import _lib
    _lib.call("kvecc_golay_h_row_masks_host", ctypes.c_void_p(masks.ctypes.data))
    assert np.array_equal(masks, oracle.golay_h_row_masks())
    assert tuple(int(m) for m in masks) == config.GOLAY_H_ROW_MASKS


def test_config_matrices():
    import torch
    from kvecc import config
    g, h = config.HAMMING74_G.int(), config.HAMMING74_H.int()
    assert ((g @ h.T) % 2).sum() == 0
    b = config.GOLAY_B_MATRIX.int()
    assert torch.equal(b, b.T) and torch.equal((b @ b) % 2, torch.eye(12, dtype=torch.int32))
    assert config.get_physical_dtype("golay") == torch.int32
    with pytest.raises(ValueError):
        config.get_codeword_bits("bch")


@pytest.mark.parametrize("ber", [1e-4, 1e-3, 1e-2, 0.05, 0.2, 0.5, 0.999, 1.0, 2.0, 1e-9,
                                 float("nan"), 0.0, -1.0, 3.3e-3])
def test_ber_threshold_is_exact(oracle, ber):
    from kvecc import _lib
    thr = _lib.load().kvecc_ber_threshold(ber)
    fber = float(np.float32(ber))
    probe = set(range(max(0, thr - 300), min(2**31, thr + 300)))
    rng = np.random.default_rng(0)
    probe |= set(rng.integers(0, 2**31, size=2000).tolist())
    probe |= {0, 1, 2**31 - 1}
    for x in probe:
        u = oracle.uint_to_uniform(x)  # fold(x) = x for x >= 0
        assert (u < fber) == (x < thr), (ber, x, thr)
        # negative words fold to ~x
        u2 = oracle.uint_to_uniform((~x) & 0xFFFFFFFF)
        assert (u2 < fber) == (x < thr)


def test_backend_registry():
    from kvecc import backends
    with pytest.raises(ValueError):
        backends.get_codec_backend("cuda-triton")
    assert "hip" in backends.available_backends()


_SKIP_VALIDATION = {"kvecc_version", "kvecc_last_error", "kvecc_device_count", "kvecc_init_device",
                    "kvecc_golay_syndrome_table_host", "kvecc_golay_h_row_masks_host",
                    "kvecc_ber_threshold", "kvecc_paged_attention_workspace"}


def _call_with(lib, name, args_t, size):
    args = []
    for t in args_t:
        if t is ctypes.c_int64:
            args.append(size)
        elif t is ctypes.c_int:
            args.append(1)
        elif t is ctypes.c_float:
            args.append(0.5)
        elif t is ctypes.c_uint8:
            args.append(0)
        else:
            args.append(None)
    return getattr(lib, name)(*args)


def test_every_entry_point_rejects_negative_sizes():
    """Argument validation precedes any device work, on every status entry point:
    negative sizes -> KVECC_EINVAL with a message naming the function."""
    from kvecc import _lib
    lib = _lib.load()
    for name, args_t in _lib.SIGNATURES.items():
        if name in _SKIP_VALIDATION or ctypes.c_int64 not in args_t:
            continue
        rc = _call_with(lib, name, args_t, -1)
        msg = lib.kvecc_last_error().decode()
        assert rc == -1, (name, rc)
        assert name[len("kvecc_"):].split("_")[0] in msg or "negative" in msg, (name, msg)


def test_host_twins_reject_null_buffers():
    """Non-empty work with NULL buffers is an error, never a crash (host twins)."""
    from kvecc import _lib
    lib = _lib.load()
    for name, args_t in _lib.SIGNATURES.items():
        if not name.startswith("kvecc_cpu_") or ctypes.c_int64 not in args_t:
            continue
        assert _call_with(lib, name, args_t, 8) == -1, name


def test_quantizers_reject_unknown_scale_rule():
    """KVECC_SCALE_* is validated on every quantizing entry point (host twins
    run here; the device entry points validate before any launch)."""
    from kvecc import _lib
    lib = _lib.load()
    x = (ctypes.c_float * 8)()
    cw = (ctypes.c_uint8 * 8)()
    sc = (ctypes.c_float * 2)()
    for rule, want in ((2, -1), (-1, -1), (1, 0), (0, 0)):
        rc = lib.kvecc_cpu_quantize_encode_rows(x, _lib.F32, _lib.CODEC_H84, rule, cw, sc, 2, 4, 1)
        assert rc == want, (rule, rc)
    assert lib.kvecc_cpu_quantize_encode_rows(x, _lib.F32, 0, 5, cw, sc, 2, 4, 1) == -1
    assert "scale rule" in lib.kvecc_last_error().decode()
    header = open(HEADER).read()
    for fn in ("kvecc_quantize_encode_rows", "kvecc_shim_write", "kvecc_cpu_quantize_encode_rows",
               "kvecc_cpu_shim_write"):
        assert "scale_rule" in header.split(fn + "(")[1].split(";")[0], fn


@pytest.mark.gpu
def test_short_or_wrong_stats_buffers_raise(gpu):
    """The kernels add into slot (workgroup % KVECC_STATS_SLOTS) of the stats
    buffer through a raw pointer: every wrapper checks the buffer (contiguous
    int64, >= KVECC_STATS_WORDS elements, on the launch device) and raises
    ValueError instead of letting a kernel write past it."""
    import torch
    from kvecc import ops
    cw = ops.hamming84_encode(torch.randint(0, 16, (4096,), dtype=torch.uint8, device=gpu))
    out = torch.empty_like(cw)
    good = ops.new_stats(gpu)
    bad = [good[:100], good.to(torch.int32), good.view(32, 16)[:, :8], ops.new_stats("cpu"),
           torch.zeros(2 * good.numel(), dtype=torch.int64, device=gpu)[::2]]
    ops.hamming84_decode_into(cw, out, None, good)
    for st in bad:
        with pytest.raises(ValueError):
            ops.hamming84_decode_into(cw, out, None, st)
    g = ops.golay_encode_rows(torch.randint(0, 16, (64, 128), dtype=torch.uint8, device=gpu))
    rows = torch.empty(64, 128, dtype=torch.uint8, device=gpu)
    with pytest.raises(ValueError):
        ops.golay_decode_rows_into(g, rows, stats=good[:16])
    pk = g.reshape(-1).view(torch.uint8).view(-1, 4)[:, :3].contiguous().view(-1)
    nib = torch.empty((3 * g.numel() + 1) // 2, dtype=torch.uint8, device=gpu)
    with pytest.raises(ValueError):
        ops.golay_decode_packed_into(pk, nib, m=g.numel(), stats=good[:16])
    torch.cuda.synchronize()
