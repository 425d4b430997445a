"""HIP backend: the reference's codec functions over torch tensors on an MI355X.

Every public function keeps the name, arguments, return convention and error
behaviour of its counterpart in ecc_codecs/triton_kernels/ (cited per
function) and dispatches to libkvecc.so through ctypes on the current HIP
stream.  There is no CPU fallback: a non-GPU tensor raises AssertionError,
exactly like the reference's ``assert x.is_cuda``.

Two layers:
  * ``*_into`` / ``*_dev`` functions: asynchronous, write into caller buffers,
    statistics accumulate in a device int64 tensor (no host sync) -- for
    pipelines, the shim and benchmarks;
  * reference-compatible wrappers: same return tuples as the reference, which
    read the statistics back to Python ints (one sync per call, as the
    reference does).
"""

from __future__ import annotations

import ctypes
import math

import threading

import torch

from . import _lib
from .config import ErrorType

_VP = ctypes.c_void_p


def _ptr(t):
    return _VP(t.data_ptr()) if t is not None else _VP(0)


def _sptr(stats, device):
    """Pointer to a statistics buffer (or NULL), validated: the kernels add at
    slot (workgroup % KVECC_STATS_SLOTS) * KVECC_STATS_STRIDE of a contiguous
    int64 buffer on the launch device, so anything shorter, of another dtype,
    strided or elsewhere would be written past or misread."""
    if stats is None:
        return _VP(0)
    if (not isinstance(stats, torch.Tensor) or stats.dtype != torch.int64 or not stats.is_contiguous()
            or stats.numel() < STATS_SLOTS * STATS_STRIDE or stats.device != torch.device(device)):
        raise ValueError(f"stats must be a contiguous int64 tensor of >= {STATS_SLOTS * STATS_STRIDE} "
                         f"elements on {device} (ops.new_stats), got "
                         f"{getattr(stats, 'dtype', type(stats))} {tuple(getattr(stats, 'shape', ()))} "
                         f"on {getattr(stats, 'device', None)}")
    return _VP(stats.data_ptr())


def _stream(device):
    return _VP(torch.cuda.current_stream(device).cuda_stream)


def _check_gpu(t, what="Input"):
    assert t.is_cuda, f"{what} must be on CUDA device"


_ready = set()


def _ensure_device(device):
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _ready:
        _lib.call("kvecc_init_device", idx)
        _ready.add(idx)
    return idx


def reserve_counter_slots(n, device=None):
    """Make n counter slots available for launches captured into HIP graphs
    (kvecc_reserve_counter_slots; each captured stream takes one slot per capture)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    _lib.call("kvecc_reserve_counter_slots", _ensure_device(dev), int(n))


def counter_slots_check(device=None):
    """(slots handed out, non-zero counter words) of a device (kvecc_counter_slots_check;
    synchronises it).  Non-zero words with no launch in flight would be a scheduling bug."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    used, nz = ctypes.c_int64(0), ctypes.c_int64(0)
    _lib.call("kvecc_counter_slots_check", _ensure_device(dev), ctypes.byref(used), ctypes.byref(nz))
    return used.value, nz.value


STATS_SLOTS = 32    # KVECC_STATS_SLOTS
STATS_STRIDE = 16   # KVECC_STATS_STRIDE (uint64 words per slot)


def new_stats(device):
    """Zeroed sharded statistics buffer (include/kvecc.h: KVECC_STATS_WORDS words)."""
    return torch.zeros(STATS_SLOTS * STATS_STRIDE, dtype=torch.int64, device=device)


def stats_totals(stats, n=2):
    """Device tensor [n] of statistic totals (sum over the slots); no host sync."""
    return stats.view(STATS_SLOTS, STATS_STRIDE)[:, :n].sum(0)


def read_stats(stats, n=2):
    """Host ints of the first n statistics (one device->host sync)."""
    return [int(v) for v in stats_totals(stats, n).tolist()]


def kernel_timer(device=None):
    """A (start, stop) pair of timing events whose handles exist, for time_next_launch."""
    evs = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    for e in evs:
        e.record(torch.cuda.current_stream(device))  # creates the underlying hipEvent_t
    return evs


def time_next_launch(start, stop):
    """Arm kvecc_time_next_launch: the next kvecc kernel launched from this thread
    stamps its own start / end into the torch.cuda.Event pair (kernel_timer());
    read them with start.elapsed_time(stop) after a sync.  No marker packets."""
    _lib.call("kvecc_time_next_launch", ctypes.c_void_p(start.cuda_event),
              ctypes.c_void_p(stop.cuda_event))


def _flat(t, dtype):
    f = t.reshape(-1)
    if f.dtype != dtype:
        f = f.to(dtype)
    return f.contiguous()


# ============================================================================
# Hamming(7,4) / Hamming(8,4)
# ============================================================================

def hamming74_encode_into(flat_in, out):
    _lib.call("kvecc_hamming74_encode", _ptr(flat_in), _ptr(out), flat_in.numel(),
              _stream(flat_in.device))
    return out


def hamming84_encode_into(flat_in, out):
    _lib.call("kvecc_hamming84_encode", _ptr(flat_in), _ptr(out), flat_in.numel(),
              _stream(flat_in.device))
    return out


def hamming74_decode_into(flat_cw, data, flag=None, stats=None):
    _lib.call("kvecc_hamming74_decode", _ptr(flat_cw), _ptr(data), _ptr(flag), flat_cw.numel(),
              _sptr(stats, flat_cw.device), _stream(flat_cw.device))
    return data


def hamming84_decode_into(flat_cw, data, error_type=None, stats=None):
    _lib.call("kvecc_hamming84_decode", _ptr(flat_cw), _ptr(data), _ptr(error_type),
              flat_cw.numel(), _sptr(stats, flat_cw.device), _stream(flat_cw.device))
    return data


def hamming74_encode(int4_values: torch.Tensor) -> torch.Tensor:
    """INT4 (uint8 low nibble) -> Hamming(7,4) codewords; hamming74_triton.py:170-201."""
    _check_gpu(int4_values)
    flat = _flat(int4_values, torch.uint8)
    out = torch.empty_like(flat)
    hamming74_encode_into(flat, out)
    return out.view(int4_values.shape)


def hamming74_decode(codewords: torch.Tensor, return_error_detected: bool = False):
    """Hamming(7,4) SEC decode; hamming74_triton.py:218-277.

    -> (decoded, (n_corrected,)) or (decoded, error_detected, (n_corrected,))
    """
    _check_gpu(codewords)
    flat = _flat(codewords, torch.uint8)
    data = torch.empty_like(flat)
    flag = torch.empty_like(flat)
    stats = new_stats(flat.device)
    hamming74_decode_into(flat, data, flag, stats)
    n = read_stats(stats, 1)[0]
    data = data.view(codewords.shape)
    flag = flag.view(codewords.shape)
    if return_error_detected:
        return data, flag, (n,)
    return data, (n,)


def hamming84_encode(int4_values: torch.Tensor) -> torch.Tensor:
    """INT4 -> Hamming(8,4) SECDED codewords; hamming84_triton.py:217-254."""
    _check_gpu(int4_values)
    flat = _flat(int4_values, torch.uint8)
    out = torch.empty_like(flat)
    hamming84_encode_into(flat, out)
    return out.view(int4_values.shape)


def hamming84_decode(codewords: torch.Tensor, return_error_types: bool = False):
    """Hamming(8,4) SECDED decode; hamming84_triton.py:281-351.

    -> (decoded, (corrected, detected)) or (decoded, error_types, (corrected, detected))
    Double errors keep their (uncorrected) data and are typed DOUBLE_DETECTED.
    """
    _check_gpu(codewords)
    flat = _flat(codewords, torch.uint8)
    data = torch.empty_like(flat)
    etype = torch.empty_like(flat)
    stats = new_stats(flat.device)
    hamming84_decode_into(flat, data, etype, stats)
    corrected, detected = read_stats(stats)
    data = data.view(codewords.shape)
    etype = etype.view(codewords.shape)
    if return_error_types:
        return data, etype, (corrected, detected)
    return data, (corrected, detected)


# ============================================================================
# Golay(24,12)
# ============================================================================

def golay_encode_into(flat_triplets, codewords, m):
    _ensure_device(flat_triplets.device)
    _lib.call("kvecc_golay_encode", _ptr(flat_triplets), _ptr(codewords), m,
              _stream(flat_triplets.device))
    return codewords


def golay_decode_into(flat_cw, triplets, counts=None, stats=None):
    _ensure_device(flat_cw.device)
    _lib.call("kvecc_golay_decode", _ptr(flat_cw), _ptr(triplets), _ptr(counts), flat_cw.numel(),
              _sptr(stats, flat_cw.device), _stream(flat_cw.device))
    return triplets


def golay_encode(triplets: torch.Tensor) -> torch.Tensor:
    """INT4 triplets [N,3] (or [3]) -> int32 codewords [N]; golay_triton.py:382-422."""
    _check_gpu(triplets)
    if triplets.dim() == 1:
        triplets = triplets.unsqueeze(0)
    n = triplets.shape[0]
    flat = _flat(triplets, torch.uint8)
    if flat.numel() < 3 * n:
        raise ValueError(f"golay_encode needs 3 values per codeword, got shape {tuple(triplets.shape)}")
    out = torch.empty(n, dtype=torch.int32, device=triplets.device)
    golay_encode_into(flat, out, n)
    return out


def golay_decode(codewords: torch.Tensor, return_error_counts: bool = False):
    """Golay(24,12) decode; golay_triton.py:425-498.

    -> (triplets [N,3], (bits_corrected, uncorrectable)) or
       (triplets, error_counts [N], (bits_corrected, uncorrectable)).
    error_count 0..3 = bits corrected, 4 = uncorrectable (data kept).
    """
    _check_gpu(codewords)
    n = codewords.numel()
    flat = _flat(codewords, torch.int32)
    trip = torch.empty(n * 3, dtype=torch.uint8, device=codewords.device)
    counts = torch.empty(n, dtype=torch.uint8, device=codewords.device)
    stats = new_stats(codewords.device)
    golay_decode_into(flat, trip, counts, stats)
    bits, unc = read_stats(stats)
    trip = trip.view(n, 3)
    if return_error_counts:
        return trip, counts, (bits, unc)
    return trip, (bits, unc)


def golay_encode_rows(nibbles: torch.Tensor) -> torch.Tensor:
    """Per-head packing of the shim (ecc_shim.py:623-682): [..., D] nibbles ->
    [..., ceil(D/3)] codewords, each row zero-padded to a multiple of 3."""
    _check_gpu(nibbles)
    d = nibbles.shape[-1]
    g = (d + 2) // 3
    flat = _flat(nibbles, torch.uint8)
    rows = flat.numel() // d if d else 0
    out = torch.empty(*nibbles.shape[:-1], g, dtype=torch.int32, device=nibbles.device)
    _ensure_device(nibbles.device)
    _lib.call("kvecc_golay_encode_rows", _ptr(flat), _ptr(out), rows, d, _stream(nibbles.device))
    return out


def golay_decode_rows(codewords: torch.Tensor, d: int, stats=None) -> torch.Tensor:
    """Inverse of golay_encode_rows: [..., ceil(d/3)] -> [..., d] nibbles."""
    _check_gpu(codewords)
    g = codewords.shape[-1]
    if g != (d + 2) // 3:
        raise ValueError(f"{g} codewords per row do not hold {d} values")
    flat = _flat(codewords, torch.int32)
    rows = flat.numel() // g if g else 0
    out = torch.empty(*codewords.shape[:-1], d, dtype=torch.uint8, device=codewords.device)
    _ensure_device(codewords.device)
    _lib.call("kvecc_golay_decode_rows", _ptr(flat), _ptr(out), rows, d, _sptr(stats, codewords.device),
              _stream(codewords.device))
    return out

def golay_encode_rows_into(nibbles: torch.Tensor, out: torch.Tensor) -> None:
    """golay_encode_rows into a caller buffer: contiguous uint8 [..., D] nibbles ->
    contiguous int32 [..., ceil(D/3)] codewords (asynchronous on the stream)."""
    _check_gpu(nibbles)
    d = nibbles.shape[-1]
    g = (d + 2) // 3
    if (nibbles.dtype != torch.uint8 or out.dtype != torch.int32 or not nibbles.is_contiguous()
            or not out.is_contiguous() or out.shape[-1] != g or out.shape[:-1] != nibbles.shape[:-1]
            or out.device != nibbles.device):
        raise ValueError("golay_encode_rows_into: contiguous uint8 [..., D] -> int32 [..., ceil(D/3)]")
    rows = nibbles.numel() // d if d else 0
    _ensure_device(nibbles.device)
    _lib.call("kvecc_golay_encode_rows", _ptr(nibbles), _ptr(out), rows, d, _stream(nibbles.device))


def golay_decode_rows_into(codewords: torch.Tensor, out: torch.Tensor, stats=None) -> None:
    """golay_decode_rows into a caller buffer: contiguous int32 [..., ceil(D/3)] ->
    contiguous uint8 [..., D]; statistics accumulate into `stats` (asynchronous)."""
    _check_gpu(codewords)
    d = out.shape[-1]
    g = (d + 2) // 3
    if (codewords.dtype != torch.int32 or out.dtype != torch.uint8 or not codewords.is_contiguous()
            or not out.is_contiguous() or codewords.shape[-1] != g or codewords.numel() // max(g, 1) * d != out.numel()
            or out.device != codewords.device):
        raise ValueError("golay_decode_rows_into: contiguous int32 [..., ceil(D/3)] -> uint8 [..., D]")
    rows = codewords.numel() // g if g else 0
    _ensure_device(codewords.device)
    _lib.call("kvecc_golay_decode_rows", _ptr(codewords), _ptr(out), rows, d, _sptr(stats, codewords.device), _stream(codewords.device))



# ============================================================================
# Fault injection
# ============================================================================

def inject_into(flat_in, out, ber, n_bits, seed=0, counts=None, stats=None, global_n=None,
                offset0=0):
    """Flat injection into `out` (may be `flat_in`); shard-aware via global_n/offset0."""
    n = flat_in.numel()
    gn = n if global_n is None else int(global_n)
    if flat_in.dtype == torch.uint8:
        name = "kvecc_inject_u8"
    elif flat_in.dtype == torch.int32:
        name = "kvecc_inject_i32"
    else:
        raise ValueError(f"Unsupported dtype: {flat_in.dtype}. Use uint8 or int32.")
    _lib.call(name, _ptr(flat_in), _ptr(out), _ptr(counts), n, int(n_bits), int(seed), float(ber),
              gn, int(offset0), _sptr(stats, flat_in.device), _stream(flat_in.device))
    return out


def inject_rows_into(flat_in, out, rows, row_len, ber, n_bits, seed_base, stats=None):
    """Per-row injection: row r uses seed_base + r and N = row_len (shim scheme)."""
    if flat_in.dtype == torch.uint8:
        name = "kvecc_inject_rows_u8"
    elif flat_in.dtype == torch.int32:
        name = "kvecc_inject_rows_i32"
    else:
        raise ValueError(f"Unsupported dtype: {flat_in.dtype}. Use uint8 or int32.")
    _lib.call(name, _ptr(flat_in), _ptr(out), int(rows), int(row_len), int(n_bits), int(seed_base),
              float(ber), _sptr(stats, flat_in.device), _stream(flat_in.device))
    return out


def inject_bit_errors_triton(data, ber, n_bits, seed=0, return_stats=False):
    """Bernoulli bit flips, bit-exact with the reference's Philox stream.

    fault_injection_triton.py:337-424.  ber <= 0 returns `data` itself.
    -> corrupted, or (corrupted, (total_flips, elements_affected))
    """
    _check_gpu(data)
    if ber <= 0:
        if return_stats:
            return data, (0, 0)
        return data
    flat = data.reshape(-1)
    if flat.dtype not in (torch.uint8, torch.int32):
        raise ValueError(f"Unsupported dtype: {flat.dtype}. Use uint8 or int32.")
    flat = flat.contiguous()
    out = torch.empty_like(flat)
    stats = new_stats(data.device) if return_stats else None
    inject_into(flat, out, ber, n_bits, seed, stats=stats)
    out = out.view(data.shape)
    if return_stats:
        flips, affected = read_stats(stats)
        return out, (flips, affected)
    return out


inject_bit_errors = inject_bit_errors_triton


def inject_bit_errors_triton_batched(data, ber, n_bits, seed=0):
    """fault_injection_triton.py:427-431 -> (corrupted, total_flips)."""
    corrupted, (total, _) = inject_bit_errors_triton(data, ber, n_bits, seed, return_stats=True)
    return corrupted, total


def inject_bit_errors_triton_vectorized(data, ber, n_bits, seed=0, return_stats=False):
    """rand4x variant (a different, also bit-exact stream); fault_injection_triton.py:434-496."""
    _check_gpu(data)
    if ber <= 0:
        if return_stats:
            return data, (0, 0)
        return data
    flat = data.reshape(-1)
    if flat.dtype == torch.uint8:
        name = "kvecc_inject_u8_vectorized"
    elif flat.dtype == torch.int32:
        name = "kvecc_inject_i32_vectorized"
    else:
        raise ValueError(f"Unsupported dtype: {flat.dtype}. Use uint8 or int32.")
    flat = flat.contiguous()
    out = torch.empty_like(flat)
    stats = new_stats(data.device) if return_stats else None
    _lib.call(name, _ptr(flat), _ptr(out), _VP(0), flat.numel(), int(n_bits), int(seed), float(ber),
              _sptr(stats, data.device), _stream(data.device))
    out = out.view(data.shape)
    if return_stats:
        flips, affected = read_stats(stats)
        return out, (flips, affected)
    return out


# ============================================================================
# Interpolation
# ============================================================================

def _seq_layout(shape, seq_dim):
    """(outer, len, inner) of the reference's sequence axis choice (:206-236)."""
    nd = len(shape)
    if nd == 1:
        return 1, shape[0], 1
    if nd == 2:  # 2-D input: rows are sequences, seq_dim is ignored
        return shape[0], shape[1], 1
    sd = seq_dim % nd
    outer = 1
    for s in shape[:sd]:
        outer *= s
    inner = 1
    for s in shape[sd + 1:]:
        inner *= s
    return outer, shape[sd], inner


def interpolate_into(q, err, out, outer, length, inner, gate=None):
    _lib.call("kvecc_interpolate", _ptr(q), _ptr(err), _ptr(out), outer, length, inner, _ptr(gate),
              _stream(q.device))
    return out


def count_ne_into(a, b, stats):
    """stats[0] += count of positions where uint8 a != b (same shapes, one device); no sync."""
    if a.dtype != torch.uint8 or b.dtype != torch.uint8 or a.numel() != b.numel() or a.device != b.device:
        raise ValueError("count_ne_into: two uint8 tensors of one size on one device")
    a, b = a.contiguous(), b.contiguous()
    _lib.call("kvecc_count_ne_u8", _ptr(a), _ptr(b), a.numel(), _sptr(stats, a.device), _stream(a.device))
    return stats


def mc_trial_into(x, codec, ber, seed, global_n, offset0, stats):
    """One Monte-Carlo trial in one launch (kvecc_mc_trial): x uint8 [outer, len,
    heads, head_dim] ground-truth nibbles -> encode -> Philox flips -> decode
    (-> interpolation along len) -> compare; stats words 0..4 += (flips,
    affected, corrected, detected, mismatches).  No host sync."""
    _check_gpu(x)
    if x.dim() != 4 or x.dtype != torch.uint8 or not x.is_contiguous():
        raise ValueError("mc_trial_into: x must be a contiguous uint8 [outer, len, heads, head_dim] tensor")
    if codec not in _lib.MC_CODECS:
        raise ValueError(f"mc_trial_into: codec {codec!r} not in {sorted(_lib.MC_CODECS)}")
    _ensure_device(x.device)
    outer, length, heads, d = x.shape
    _lib.call("kvecc_mc_trial", _ptr(x), outer, length, heads, d, _lib.MC_CODECS[codec], float(ber), int(seed),
              int(global_n), int(offset0), _sptr(stats, x.device), _stream(x.device))
    return stats


def stats_fold_into(stats, nbuf, nwords, dst):
    """dst[b, w] += statistic w of buffer b (nbuf buffers of KVECC_STATS_WORDS
    words back to back), then zero the buffers (kvecc_stats_fold); one launch."""
    if stats.dtype != torch.int64 or not stats.is_contiguous() or stats.numel() < nbuf * STATS_SLOTS * STATS_STRIDE:
        raise ValueError("stats_fold_into: stats must hold nbuf contiguous int64 statistics buffers")
    if dst.dtype != torch.int64 or dst.dim() != 2 or dst.shape[0] < nbuf or dst.shape[1] < nwords or dst.stride(1) != 1:
        raise ValueError("stats_fold_into: dst must be int64 [>= nbuf, >= nwords] with unit column stride")
    if dst.device != stats.device:
        raise ValueError("stats_fold_into: stats and dst on different devices")
    _lib.call("kvecc_stats_fold", _ptr(stats), int(nbuf), int(nwords), _ptr(dst), dst.stride(0),
              _stream(stats.device))
    return dst


def any_equal(x, value, flag=None):
    """Device int32 flag = any(x == value), no host sync."""
    if flag is None:
        flag = torch.empty(1, dtype=torch.int32, device=x.device)
    _lib.call("kvecc_any_equal_u8", _ptr(x), x.numel(), int(value), _ptr(flag), _stream(x.device))
    return flag


def interpolate_double_errors(q, error_type, original_shape=None, seq_dim=-1):
    """Replace DOUBLE_DETECTED values by the rounded mean of their sequence
    neighbours; interpolation_triton.py:162-265.

    The no-double fast path (return q unchanged) is decided on the device: for
    uint8 q one pass (kvecc_interpolate_auto) with no host sync and no separate
    scan of error_type; other dtypes sync once (the result dtype depends on the
    branch).
    """
    _check_gpu(q)
    _check_gpu(error_type, "Error type")
    assert q.shape == error_type.shape, "Shape mismatch between q and error_type"
    if q.numel() == 0:
        return q.clone()
    err = _flat(error_type, torch.uint8)
    outer, length, inner = _seq_layout(tuple(q.shape), seq_dim)
    if q.dtype == torch.uint8:
        qf = _flat(q, torch.uint8)
        out = torch.empty_like(qf)
        interpolate_auto_into(qf, err, out, outer, length, inner)
        return out.view(q.shape)
    flag = any_equal(err, ErrorType.DOUBLE_DETECTED)
    if int(flag.item()) == 0:
        return q.clone()
    qf = _flat(q, torch.uint8)
    out = torch.empty_like(qf)
    interpolate_into(qf, err, out, outer, length, inner)
    return out.view(q.shape)


class _EpochFlags:
    """Per-(device, stream) int32[2] flag words for kvecc_interpolate_auto and
    their call counter: each call stamps a fresh epoch, so the words never need
    zeroing (a stream orders its calls, so reuse on one stream is safe)."""

    def __init__(self):
        self._bufs = {}
        self._lock = threading.Lock()

    def next(self, device):
        if torch.cuda.is_current_stream_capturing():
            # a captured call replays with the epoch it was captured with, so
            # stale words from the previous replay would read as "seen": give
            # the graph its own words, zeroed by a captured fill on every replay
            return torch.zeros(2, dtype=torch.int32, device=device), 1
        key = (device, torch.cuda.current_stream(device).cuda_stream)
        with self._lock:
            buf, epoch = self._bufs.get(key, (None, 0))
            if buf is None or epoch >= 0x7FFFFFFF:
                buf, epoch = torch.zeros(2, dtype=torch.int32, device=device), 0
            epoch += 1
            self._bufs[key] = (buf, epoch)
        return buf, epoch


_EPOCH_FLAGS = _EpochFlags()


def interpolate_auto_into(q, err, out, outer, length, inner):
    """kvecc_interpolate_auto: interpolation and the no-double fast path in one
    pass.  Returns (flags, epoch): flags[k] == epoch <=> (any err == 2, any q > 15)."""
    flags, epoch = _EPOCH_FLAGS.next(q.device)
    _lib.call("kvecc_interpolate_auto", _ptr(q), _ptr(err), _ptr(out), outer, length, inner,
              _ptr(flags), epoch, _stream(q.device))
    return flags, epoch


def interpolate_double_errors_1d(q, error_type):
    return interpolate_double_errors(q, error_type, seq_dim=-1)


def interpolate_double_errors_autotuned(q, error_type, original_shape=None, seq_dim=-1):
    """Same result as interpolate_double_errors (the reference autotunes Triton
    block sizes, :272-350; the HIP kernel's geometry is fixed per layout)."""
    return interpolate_double_errors(q, error_type, original_shape, seq_dim)


# ============================================================================
# Fused quantize + encode / decode + dequantize
# ============================================================================

_DT = {torch.float32: _lib.F32, torch.float16: _lib.F16, torch.bfloat16: _lib.BF16}

# Row-scale rule when the caller names none: the reference's `abs_max / 7.0` as
# torch evaluates it on this backend's device (GPU tensors: abs_max * RN(1/7);
# kvecc.h KVECC_SCALE_*).  Pass scale_rule="div7" to reproduce the reference run
# on the CPU.
DEFAULT_SCALE_RULE = "mul_inv7"


def quantize_encode_rows_into(x2d, codec_code, cw, scales, scale_rule=None):
    if x2d.dtype not in _DT:
        raise TypeError(f"unsupported input dtype {x2d.dtype}")
    rows, d = x2d.shape
    _lib.call("kvecc_quantize_encode_rows", _ptr(x2d), _DT[x2d.dtype], int(codec_code),
              _lib.scale_rule_code(scale_rule, DEFAULT_SCALE_RULE), _ptr(cw),
              _ptr(scales), rows, d, _stream(x2d.device))
    return cw, scales


def _fused_quantize_encode(input_tensor, codec_code, scale_rule=None):
    _check_gpu(input_tensor)
    shape = input_tensor.shape
    d = shape[-1]
    x = input_tensor.reshape(-1, d).contiguous()
    rows = x.shape[0]
    cw = torch.empty(rows, d, dtype=torch.uint8, device=input_tensor.device)
    scales = torch.empty(rows, dtype=torch.float32, device=input_tensor.device)
    quantize_encode_rows_into(x, codec_code, cw, scales, scale_rule)
    if input_tensor.dim() == 1:
        return cw.squeeze(0), scales
    return cw.view(shape), scales.view(shape[:-1])


def fused_quantize_encode_hamming84(input_tensor, scale_rule=None):
    """Row absmax INT4 quantization + Hamming(8,4) encode in one kernel;
    fused_kernels.py:97-160 (matches the shim's torch rounding exactly)."""
    return _fused_quantize_encode(input_tensor, _lib.CODEC_H84, scale_rule)


def fused_quantize_encode_hamming74(input_tensor, scale_rule=None):
    """fused_kernels.py:222-269 with Hamming(7,4)."""
    return _fused_quantize_encode(input_tensor, _lib.CODEC_H74, scale_rule)


def quantize_rows(input_tensor, scale_rule=None):
    """INT4 quantization only (codec 'int4'): -> (nibbles uint8, scales f32)."""
    return _fused_quantize_encode(input_tensor, _lib.CODEC_NONE, scale_rule)


def decode_dequant_h84_into(cw2d, scales, out, zero_doubles=True, stats=None):
    rows, d = cw2d.shape
    _lib.call("kvecc_decode_dequant_h84_rows", _ptr(cw2d), _ptr(scales), _ptr(out), _DT[out.dtype],
              rows, d, int(bool(zero_doubles)), _sptr(stats, cw2d.device), _stream(cw2d.device))
    return out


def fused_decode_dequantize_hamming84(codewords, scales, output_dtype=torch.float32):
    """Hamming(8,4) decode + dequantize; fused_kernels.py:372-437.

    Double-error values become 0 before dequantization (:344).
    -> (dequantized, errors_corrected)
    """
    _check_gpu(codewords)
    _check_gpu(scales, "Scales")
    shape = codewords.shape
    d = shape[-1]
    cw = codewords.reshape(-1, d).contiguous()
    sc = scales.reshape(-1).to(torch.float32).contiguous()
    dtype = output_dtype if output_dtype in _DT else torch.float32
    out = torch.empty(cw.shape, dtype=dtype, device=codewords.device)
    stats = new_stats(codewords.device)
    decode_dequant_h84_into(cw, sc, out, True, stats)
    corrected = read_stats(stats, 1)[0]
    out = out.squeeze(0) if codewords.dim() == 1 else out.view(shape)
    if output_dtype != dtype:
        out = out.to(output_dtype)
    return out, corrected


# ============================================================================
# ECC shim: paged KV-cache write / read (one launch each)
# ============================================================================

SHIM_CODECS = {"int4": _lib.CODEC_NONE, "hamming74": _lib.CODEC_H74, "hamming84": _lib.CODEC_H84,
               "golay": _lib.CODEC_GOLAY, "golay_packed": _lib.CODEC_GOLAY_PACKED}


def shim_write(k, v, manager, layer, codec, n_bits, inject, ber, seed0, seq_id=0,
               scale_rule=None):
    """ECCBackend.write for one layer (ecc_shim.py:557-721): K, V [batch, seq,
    hkv*d] or [batch, seq, hkv, d] -> quantize, encode, per-row inject, scatter
    into manager's caches.  Strided views whose head rows are contiguous are read
    in place (kvecc_shim_write_strided), anything else is made contiguous."""
    shim_write_tensors(k, v, manager.k_cache, manager.v_cache, manager.k_scales, manager.v_scales,
                       manager.block_table[seq_id], manager.num_layers, manager.block_size,
                       manager.num_kv_heads, manager.head_dim, layer, codec, n_bits, inject, ber, seed0,
                       scale_rule)


def shim_write_tensors(k, v, k_cache, v_cache, k_scales, v_scales, table, num_layers, block_size, hkv, d,
                       layer, codec, n_bits, inject, ber, seed0, scale_rule=None):
    """shim_write on the cache tensors themselves (the torch.ops.kvecc.shim_write
    kernel): table = the sequence's block-table row, int32 [max_blocks]."""
    batch, seq = k.shape[0], k.shape[1]
    if k.dtype not in _DT or v.dtype != k.dtype:
        raise TypeError(f"unsupported K/V dtype {k.dtype}/{v.dtype}")
    k4 = _head_rows(k, batch, seq, hkv, d)
    v4 = _head_rows(v, batch, seq, hkv, d)
    _lib.call("kvecc_shim_write_strided", _ptr(k4), _ptr(v4), k4.stride(0), k4.stride(1),
              k4.stride(2), v4.stride(0), v4.stride(1), v4.stride(2), _DT[k.dtype], batch, seq,
              hkv, d, SHIM_CODECS[codec], _lib.scale_rule_code(scale_rule, DEFAULT_SCALE_RULE),
              int(n_bits), int(bool(inject)), float(ber), int(seed0), _ptr(k_cache), _ptr(v_cache),
              _ptr(k_scales), _ptr(v_scales), _ptr(table), int(num_layers), int(block_size), int(layer),
              _stream(k.device))


def _head_rows(x, batch, seq, hkv, d):
    """[batch, seq, hkv, d] view of x with unit element stride and head stride
    >= d (a copy only when no such view exists)."""
    try:
        x4 = x.view(batch, seq, hkv, d)
    except RuntimeError:
        x4 = None
    if x4 is None or x4.stride(3) != 1 or x4.stride(2) < d or min(x4.stride()) < 0:
        x4 = x.reshape(batch, seq, hkv, d).contiguous()
    return x4


def shim_read(manager, layer, ctx, codec, interp, out_dtype, stats=None, seq_id=0):
    """ECCBackend.attend decode side (ecc_shim.py:990-1071) -> K, V [hkv, ctx, d]
    in out_dtype (decode, optional H84 interpolation along ctx, dequantize)."""
    return shim_read_tensors(manager.k_cache, manager.v_cache, manager.k_scales, manager.v_scales,
                             manager.block_table[seq_id], ctx, manager.num_kv_heads, manager.head_dim,
                             manager.num_layers, manager.block_size, layer, codec, interp, out_dtype, stats)


def shim_read_tensors(k_cache, v_cache, k_scales, v_scales, table, ctx, hkv, d, num_layers, block_size,
                      layer, codec, interp, out_dtype, stats=None):
    """shim_read on the cache tensors themselves (the torch.ops.kvecc.shim_read kernel)."""
    dev = k_cache.device
    shape = (hkv, ctx, d)
    k_out = torch.empty(shape, dtype=out_dtype, device=dev)
    v_out = torch.empty(shape, dtype=out_dtype, device=dev)
    _lib.call("kvecc_shim_read", _ptr(k_cache), _ptr(v_cache), _ptr(k_scales), _ptr(v_scales), _ptr(table),
              int(ctx), int(hkv), int(d), int(num_layers), int(block_size), int(layer), SHIM_CODECS[codec],
              int(bool(interp)), _ptr(k_out), _ptr(v_out), _DT[out_dtype], _sptr(stats, dev), _stream(dev))
    return k_out, v_out


_SHIM_CACHE_DT = {"int4": torch.uint8, "hamming74": torch.uint8, "hamming84": torch.uint8,
                  "golay": torch.int32, "golay_packed": torch.uint8}


def _check_shim_read_args(k_cache, v_cache, k_scales, v_scales, block_table, ctx, head_dim, layer, codec,
                          out_dtype, stats, out):
    """Validate a batched shim read (both backends): cache dtype per codec and
    geometry, scales [blocks, layers, hkv, block_size] fp32, the block table,
    a caller-supplied ``out`` pair ([B, hkv, ctx, head_dim], out_dtype,
    contiguous), and one device for every tensor -- a mismatch raises
    ValueError instead of reading or writing past an allocation.
    Returns (batch, layers, hkv, block_size)."""
    if codec not in _SHIM_CACHE_DT:
        raise ValueError(f"shim codec {codec!r} (int4, hamming74, hamming84, golay or golay_packed)")
    if out_dtype not in _DT:
        raise ValueError(f"out_dtype must be fp32/fp16/bf16, got {out_dtype}")
    if k_cache.dim() != 4 or k_cache.shape != v_cache.shape:
        raise ValueError("k_cache / v_cache must share one [blocks, layers, kv_heads, row] shape")
    nb, nl, hkv, row = k_cache.shape
    for name, c in (("k_cache", k_cache), ("v_cache", v_cache)):
        if c.dtype != _SHIM_CACHE_DT[codec]:
            raise ValueError(f"{codec} {name} must be {_SHIM_CACHE_DT[codec]}, got {c.dtype}")
    if head_dim < 1:
        raise ValueError(f"head_dim must be positive, got {head_dim}")
    per = {"golay": (head_dim + 2) // 3, "golay_packed": (3 * ((head_dim + 2) // 3) + 3) // 4 * 4}.get(
        codec, head_dim)
    if row % per:
        raise ValueError(f"cache rows of {row} words do not hold whole token rows of {per}")
    bs = row // per
    if not 0 <= int(layer) < nl:
        raise ValueError(f"layer {layer} outside the cache's {nl} layers")
    if block_table.dim() != 2 or block_table.dtype != torch.int32:
        raise ValueError("block_table must be a contiguous int32 [B, max_blocks] tensor")
    if block_table.shape[1] * bs < ctx:
        raise ValueError(f"block_table covers {block_table.shape[1] * bs} tokens < ctx {ctx}")
    for name, sc in (("k_scales", k_scales), ("v_scales", v_scales)):
        if sc.shape != (nb, nl, hkv, bs) or sc.dtype != torch.float32:
            raise ValueError(f"{name} must be float32 [{nb}, {nl}, {hkv}, {bs}], got "
                             f"{tuple(sc.shape)} {sc.dtype}")
    batch = block_table.shape[0]
    tensors = [("k_cache", k_cache), ("v_cache", v_cache), ("k_scales", k_scales), ("v_scales", v_scales),
               ("block_table", block_table)]
    if out is not None:
        shape = (batch, hkv, ctx, head_dim)
        for name, o in zip(("k_out", "v_out"), out):
            if tuple(o.shape) != shape or o.dtype != out_dtype:
                raise ValueError(f"{name} must be {out_dtype} {list(shape)}, got {o.dtype} {list(o.shape)}")
            tensors.append((name, o))
    for name, t in tensors:
        if t.device != k_cache.device:
            raise ValueError(f"{name} is on {t.device}, k_cache on {k_cache.device}")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
    if stats is not None and stats.device != k_cache.device:
        raise ValueError(f"stats is on {stats.device}, k_cache on {k_cache.device}")
    return batch, nl, hkv, bs


def shim_read_batch(k_cache, v_cache, k_scales, v_scales, block_table, ctx, head_dim, layer, codec,
                    out_dtype, stats=None, interp=False, out=None):
    """The shim's fused read (gather -> decode -> dequantize, ecc_shim.py:990-1071)
    for every sequence of a paged cache at once: block_table [B, max_blocks]
    int32 (row b = sequence b), caches [blocks, layers, hkv, block_size * P]
    -> (K, V) [B, hkv, ctx, head_dim] in out_dtype (kvecc_shim_read_batch)."""
    _check_gpu(k_cache)
    batch, nl, hkv, bs = _check_shim_read_args(k_cache, v_cache, k_scales, v_scales, block_table, ctx,
                                               head_dim, layer, codec, out_dtype, stats, out)
    shape = (batch, hkv, ctx, head_dim)
    if out is None:
        out = (torch.empty(shape, dtype=out_dtype, device=k_cache.device),
               torch.empty(shape, dtype=out_dtype, device=k_cache.device))
    k_out, v_out = out
    _lib.call("kvecc_shim_read_batch", _ptr(k_cache), _ptr(v_cache), _ptr(k_scales), _ptr(v_scales),
              _ptr(block_table), block_table.shape[1], batch, int(ctx), hkv, head_dim, nl, bs,
              int(layer), SHIM_CODECS[codec], int(bool(interp)), _ptr(k_out), _ptr(v_out),
              _DT[out_dtype], _sptr(stats, k_cache.device), _stream(k_cache.device))
    return k_out, v_out


# ============================================================================
# Paged decode attention with inline ECC decode
# ============================================================================

_ATTN_ROW_WORDS = {"hamming84": lambda d: d, "golay": lambda d: (d + 2) // 3,
                   "golay_packed": lambda d: (3 * ((d + 2) // 3) + 3) // 4 * 4}  # KVECC_GOLAY_PACKED_ROW
_ATTN_CACHE_DT = {"hamming84": torch.uint8, "golay": torch.int32, "golay_packed": torch.uint8}
_attn_ws = {}  # (device index, stream) -> float32 workspace, grown on demand
_attn_ws_retired = []  # outgrown workspaces stay alive: a captured HIP graph may still name them


def _attn_workspace(device, n):
    key = (device.index, torch.cuda.current_stream(device).cuda_stream)
    ws = _attn_ws.get(key)
    if ws is None or ws.numel() < n:
        if ws is not None:
            _attn_ws_retired.append(ws)
        ws = torch.empty(max(n, 1), dtype=torch.float32, device=device)
        _attn_ws[key] = ws
    return ws


def _check_attention_args(query, k_cache, v_cache, block_table, context_lens, k_scales, v_scales,
                          out, block_size, codec):
    if codec not in _ATTN_CACHE_DT:
        raise ValueError(f"paged attention codec {codec!r} (hamming84, golay or golay_packed)")
    if query.dim() != 3 or query.dtype not in _DT:
        raise ValueError(f"query must be [B, H, D] fp32/fp16/bf16, got {tuple(query.shape)} {query.dtype}")
    batch, heads, head_dim = query.shape
    if k_cache.dim() != 4 or k_cache.shape != v_cache.shape:
        raise ValueError("k_cache / v_cache must share one [blocks, layers, kv_heads, row] shape")
    nb, nl, kvh, row = k_cache.shape
    per = _ATTN_ROW_WORDS[codec](head_dim)
    for name, c in (("k_cache", k_cache), ("v_cache", v_cache)):
        if c.dtype != _ATTN_CACHE_DT[codec]:
            raise ValueError(f"{codec} {name} must be {_ATTN_CACHE_DT[codec]}, got {c.dtype}")
    if row != block_size * per:
        raise ValueError(f"{codec} cache rows hold {row} words, expected block_size*{per} = "
                         f"{block_size * per}")
    if kvh < 1 or heads % kvh:
        raise ValueError(f"{heads} query heads not a multiple of {kvh} kv heads")
    if block_table.dim() != 2 or block_table.shape[0] != batch or block_table.dtype != torch.int32:
        raise ValueError("block_table must be int32 [B, max_blocks]")
    if context_lens.shape != (batch,) or context_lens.dtype != torch.int32:
        raise ValueError("context_lens must be int32 [B]")
    for name, sc in (("k_scales", k_scales), ("v_scales", v_scales)):
        if sc.shape != (nb, nl, kvh, block_size) or sc.dtype != torch.float32:
            raise ValueError(f"{name} must be float32 [{nb}, {nl}, {kvh}, {block_size}], got "
                             f"{tuple(sc.shape)} {sc.dtype}")
    if out.shape != query.shape or out.dtype not in _DT:
        raise ValueError("out must match query's [B, H, D]")
    for name, t in (("query", query), ("k_cache", k_cache), ("v_cache", v_cache),
                    ("block_table", block_table), ("context_lens", context_lens),
                    ("k_scales", k_scales), ("v_scales", v_scales), ("out", out)):
        if t.device != query.device:
            raise ValueError(f"{name} is on {t.device}, query on {query.device}")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")


def paged_attention_into(query, k_cache, v_cache, block_table, context_lens, k_scales, v_scales,
                         out, layer_idx, block_size, sm_scale, codec, max_context_len=0):
    """kvecc_paged_attention on [B, H, D] query / out (see include/kvecc.h).

    Every argument is validated (dtypes, geometry against codec and block_size,
    contiguity, one device): a mismatch raises ValueError instead of reading
    past an allocation.  The split workspace is cached per (device, stream).
    ``out`` may differ in dtype from ``query`` only as the kernel allows (the
    query dtype is the output dtype)."""
    _check_gpu(query, "Query")
    _check_attention_args(query, k_cache, v_cache, block_table, context_lens, k_scales, v_scales,
                          out, block_size, codec)
    if out.dtype != query.dtype:
        raise ValueError(f"out dtype {out.dtype} != query dtype {query.dtype}")
    batch, heads, head_dim = query.shape
    num_blocks, num_layers, kv_heads, _ = k_cache.shape
    max_blocks = block_table.shape[1]
    mcl = int(max_context_len) if max_context_len and max_context_len > 0 else max_blocks * block_size
    ws_n = _lib.load().kvecc_paged_attention_workspace(batch, heads, head_dim, mcl)
    ws = _attn_workspace(query.device, ws_n)
    _lib.call("kvecc_paged_attention", _ptr(query), _DT[query.dtype], _ptr(k_cache), _ptr(v_cache),
              _ptr(block_table), _ptr(context_lens), _ptr(k_scales), _ptr(v_scales), _ptr(out),
              batch, heads, kv_heads, head_dim, num_blocks, num_layers, int(layer_idx), int(block_size),
              max_blocks, mcl, float(sm_scale), SHIM_CODECS[codec], _ptr(ws), ws.numel(),
              _stream(query.device))
    return out


def _conform(t, dtype):
    """t itself when it already has dtype and is contiguous (no copy)."""
    if t.dtype != dtype:
        t = t.to(dtype)
    return t if t.is_contiguous() else t.contiguous()


def paged_attention_ecc(query, k_cache, v_cache, block_table, context_lens, k_scales, layer_idx,
                        block_size, sm_scale=None, codec="hamming84", syndrome_table=None,
                        use_tiled=False, block_m=4, v_scales=None):
    """Single-token paged attention over the ECC cache; attention_ecc.py:620-780.

    query [B, H, D]; caches [blocks, layers, Hkv, block_size * P]; block_table
    [B, max_blocks] int32; context_lens [B] int32.  -> [B, H, D] in query's
    dtype.  As in the reference: v_scales defaults to k_scales; the "golay"
    codec reproduces reference_attention_ecc (:783-909), which dequantizes K
    and V with k_scales and returns fp32.  syndrome_table is accepted for
    signature compatibility (the table lives on the device).  use_tiled with
    block_size >= block_m selects the reference's tiled kernel (:430-617, :693):
    the same attention (one split kernel computes both), except that a context
    with no valid token gives 0 there instead of the default kernel's -8.0
    (tiled_empty_to_zero).
    """
    _check_gpu(query, "Query")
    if codec not in ("hamming84", "golay"):
        raise ValueError(f"Unknown codec: {codec}")
    if codec == "hamming84":
        assert k_cache.dtype == torch.uint8, "Hamming84 K cache must be uint8"
        assert v_cache.dtype == torch.uint8, "Hamming84 V cache must be uint8"
    else:
        assert k_cache.dtype == torch.int32, "Golay K cache must be int32"
        assert v_cache.dtype == torch.int32, "Golay V cache must be int32"
        v_scales = k_scales  # reference_attention_ecc uses one scale tensor for K and V
    if v_scales is None:
        v_scales = k_scales
    head_dim = query.shape[-1]
    if sm_scale is None:
        sm_scale = 1.0 / math.sqrt(head_dim)
    q = query.contiguous()
    out_dtype = torch.float32 if codec == "golay" else q.dtype
    if q.dtype not in _DT:
        raise TypeError(f"unsupported query dtype {q.dtype}")
    if out_dtype != q.dtype:
        q = q.to(out_dtype)
    out = torch.empty(q.shape, dtype=out_dtype, device=q.device)
    paged_attention_into(q, _conform(k_cache, k_cache.dtype), _conform(v_cache, v_cache.dtype),
                         _conform(block_table, torch.int32), _conform(context_lens, torch.int32),
                         _conform(k_scales, torch.float32), _conform(v_scales, torch.float32),
                         out, layer_idx, block_size, sm_scale, codec)
    if codec == "hamming84" and use_tiled and block_size >= block_m:
        tiled_empty_to_zero(out, block_table, context_lens, block_size)
    return out


def tiled_empty_to_zero(out, block_table, context_lens, block_size):
    """The reference's tiled H84 kernel ends with ``l_i > 0 ? acc / l_i : 0``
    (attention_ecc.py:614): a sequence with no valid token -- no block j with
    j * block_size < context_len and block_table[b, j] >= 0 (:497-510) -- is 0,
    where the default kernel's masked rows give -8.0.  In place on `out`."""
    nb = block_table.shape[1]
    start = torch.arange(nb, device=block_table.device, dtype=torch.int64) * block_size
    valid = (start[None, :] < context_lens.to(torch.int64)[:, None]) & (block_table >= 0)
    out.masked_fill_(~valid.any(dim=1)[:, None, None], 0.0)


# ============================================================================
# Packed Golay storage (native layout; include/kvecc.h "Packed Golay storage")
# ============================================================================

def pack_nibbles(values: torch.Tensor) -> torch.Tensor:
    """INT4 values (uint8, low nibble) -> bytes, two per byte, low nibble first."""
    flat = values.reshape(-1).to(torch.uint8)
    if flat.numel() % 2:
        flat = torch.cat([flat, flat.new_zeros(1)])
    pairs = flat.view(-1, 2) & 0xF
    return (pairs[:, 0] | (pairs[:, 1] << 4)).contiguous()


def unpack_nibbles(packed: torch.Tensor, n: int) -> torch.Tensor:
    """Inverse of pack_nibbles: the first n values as uint8."""
    p = packed.reshape(-1)
    return torch.stack([p & 0xF, p >> 4], dim=1).reshape(-1)[:n].contiguous()


def _check_packed_bufs(name, m, *bufs):
    """Raw-pointer packed entry points: every buffer a contiguous uint8 tensor on
    the first one's GPU, holding at least the bytes the kernel touches for m
    units (the kernels take only pointers, so a short buffer would be overrun)."""
    dev = bufs[0][0].device
    _check_gpu(bufs[0][0])
    if m < 0:
        raise ValueError(f"{name}: negative count {m}")
    for t, need, what in bufs:
        if t is None:
            continue
        if t.dtype != torch.uint8 or not t.is_contiguous() or t.device != dev:
            raise ValueError(f"{name}: {what} must be a contiguous uint8 tensor on {dev}")
        if t.numel() < need:
            raise ValueError(f"{name}: {what} holds {t.numel()} bytes, needs {need}")


def golay_encode_packed_into(nibbles, codewords, m):
    """Asynchronous packed encode into caller buffers (device pointers, stream)."""
    m = int(m)
    _check_packed_bufs("golay_encode_packed_into", m, (nibbles, (3 * m + 1) // 2, "nibbles"),
                       (codewords, 3 * m, "codewords"))
    _lib.call("kvecc_golay_encode_packed", _ptr(nibbles), _ptr(codewords), int(m),
              _stream(nibbles.device))
    return codewords


def golay_decode_packed_into(codewords, nibbles, uncorrectable=None, m=None, stats=None):
    """Asynchronous packed decode into caller buffers; statistics stay on the device."""
    m = codewords.numel() // 3 if m is None else int(m)
    _check_packed_bufs("golay_decode_packed_into", m, (codewords, 3 * m, "codewords"),
                       (nibbles, (3 * m + 1) // 2, "nibbles"), (uncorrectable, (m + 7) // 8, "uncorrectable"))
    _lib.call("kvecc_golay_decode_packed", _ptr(codewords), _ptr(nibbles), _ptr(uncorrectable), m,
              _sptr(stats, codewords.device), _stream(codewords.device))
    return nibbles


def golay_encode_packed(nibbles: torch.Tensor, m: int) -> torch.Tensor:
    """m codewords of the packed nibble stream (3 values each) -> 3m codeword bytes."""
    _check_gpu(nibbles)
    nib = nibbles.reshape(-1)
    if nib.dtype != torch.uint8 or nib.numel() < (3 * m + 1) // 2:
        raise ValueError(f"need {(3 * m + 1) // 2} packed uint8 nibble bytes for {m} codewords")
    nib = nib.contiguous()
    out = torch.empty(3 * m, dtype=torch.uint8, device=nib.device)
    _ensure_device(nib.device)
    _lib.call("kvecc_golay_encode_packed", _ptr(nib), _ptr(out), int(m), _stream(nib.device))
    return out


def golay_decode_packed(codewords: torch.Tensor, m: int, return_uncorrectable: bool = False,
                        stats=None):
    """3m codeword bytes -> packed nibbles (ceil(3m/2) bytes), (bits_corrected,
    uncorrectable) [, uncorrectable bitmask ceil(m/8) bytes]."""
    _check_gpu(codewords)
    cw = codewords.reshape(-1)
    if cw.dtype != torch.uint8 or cw.numel() < 3 * m:
        raise ValueError(f"need {3 * m} uint8 codeword bytes for {m} codewords")
    cw = cw.contiguous()
    dev = cw.device
    nib = torch.empty((3 * m + 1) // 2, dtype=torch.uint8, device=dev)
    flags = torch.empty((m + 7) // 8, dtype=torch.uint8, device=dev) if return_uncorrectable else None
    st = new_stats(dev) if stats is None else stats
    _ensure_device(dev)
    _lib.call("kvecc_golay_decode_packed", _ptr(cw), _ptr(nib), _ptr(flags), int(m), _sptr(st, dev),
              _stream(dev))
    if stats is not None:
        return (nib, flags) if return_uncorrectable else nib
    bits, unc = read_stats(st)
    if return_uncorrectable:
        return nib, flags, (bits, unc)
    return nib, (bits, unc)


def pack_error_types(types: torch.Tensor) -> torch.Tensor:
    """ErrorType bytes (0..3) -> 2 bits per value, value j at bits 2*(j%4) of byte j/4."""
    flat = types.reshape(-1).to(torch.uint8)
    pad = (4 - flat.numel() % 4) % 4
    if pad:
        flat = torch.cat([flat, flat.new_zeros(pad)])
    q = (flat.view(-1, 4) & 3).to(torch.int32)
    return (q[:, 0] | q[:, 1] << 2 | q[:, 2] << 4 | q[:, 3] << 6).to(torch.uint8)


def hamming84_encode_packed_into(nibbles, codewords, n):
    n = int(n)
    _check_packed_bufs("hamming84_encode_packed_into", n, (nibbles, (n + 1) // 2, "nibbles"),
                       (codewords, n, "codewords"))
    _lib.call("kvecc_hamming84_encode_packed", _ptr(nibbles), _ptr(codewords), int(n),
              _stream(nibbles.device))
    return codewords


def hamming84_decode_packed_into(codewords, nibbles, error_types=None, n=None, stats=None):
    n = codewords.numel() if n is None else int(n)
    _check_packed_bufs("hamming84_decode_packed_into", n, (codewords, n, "codewords"),
                       (nibbles, (n + 1) // 2, "nibbles"), (error_types, (n + 3) // 4, "error_types"))
    _lib.call("kvecc_hamming84_decode_packed", _ptr(codewords), _ptr(nibbles), _ptr(error_types), n,
              _sptr(stats, codewords.device), _stream(codewords.device))
    return nibbles


def hamming84_encode_packed(nibbles: torch.Tensor, n: int) -> torch.Tensor:
    """n values of a packed nibble stream -> n Hamming(8,4) codeword bytes."""
    _check_gpu(nibbles)
    nib = nibbles.reshape(-1)
    if nib.dtype != torch.uint8 or nib.numel() < (n + 1) // 2:
        raise ValueError(f"need {(n + 1) // 2} packed uint8 nibble bytes for {n} values")
    nib = nib.contiguous()
    out = torch.empty(n, dtype=torch.uint8, device=nib.device)
    return hamming84_encode_packed_into(nib, out, n)


def hamming84_decode_packed(codewords: torch.Tensor, return_error_types: bool = False):
    """Codeword bytes -> packed nibbles, (corrected, detected) [, packed 2-bit types]."""
    _check_gpu(codewords)
    cw = codewords.reshape(-1).to(torch.uint8).contiguous()
    n = cw.numel()
    nib = torch.empty((n + 1) // 2, dtype=torch.uint8, device=cw.device)
    et = torch.empty((n + 3) // 4, dtype=torch.uint8, device=cw.device) if return_error_types else None
    st = new_stats(cw.device)
    hamming84_decode_packed_into(cw, nib, et, n, st)
    corrected, detected = read_stats(st)
    if return_error_types:
        return nib, et, (corrected, detected)
    return nib, (corrected, detected)
