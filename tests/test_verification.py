"""evaluation/verification.py's checks (GF(2) code properties + exhaustive
single/double-bit error statistics) as tests, on the host backend (CPU) and
the HIP backend (GPU).  The error statistics are recomputed independently
with the oracle's decoders, one corrupted word at a time, as the reference
loops (verification.py:215-349)."""

from itertools import combinations

import pytest
import torch


def _oracle_amplification(oracle, h84):
    import numpy as np
    nb = 8 if h84 else 7
    enc = oracle.hamming84_encode if h84 else oracle.hamming74_encode
    dec = oracle.hamming84_decode if h84 else oracle.hamming74_decode
    pop = lambda x: bin(x).count("1")  # noqa: E731
    single_ok = det = mis = 0
    d1 = d2 = 0
    for v in range(16):
        cw = int(enc(np.array([v], np.uint8))[0])
        for b in range(nb):
            c = cw ^ (1 << b)
            out = dec(np.array([c], np.uint8))
            d = int(out[0][0])
            single_ok += d == v
            d1 += pop(v ^ d) - pop(v ^ (c & 0xF))
        for b1, b2 in combinations(range(nb), 2):
            c = cw ^ (1 << b1) ^ (1 << b2)
            out = dec(np.array([c], np.uint8))
            d = int(out[0][0])
            delta = pop(v ^ d) - pop(v ^ (c & 0xF))
            d2 += delta
            if (h84 and int(out[1][0]) == 2) or delta <= 0:
                det += 1
            else:
                mis += 1
    return single_ok, det, mis, d1 / (16 * nb), d2 / (16 * nb * (nb - 1) // 2)


def _check(device, oracle):
    from kvecc.verification import format_verification_report, run_all_verifications
    reports = run_all_verifications(device)
    for name, r in reports.items():
        assert r.all_passed, format_verification_report(r)
        assert r.null_space.syndrome_zero_rate == 1.0 and r.orthogonality.is_orthogonal
        assert r.rank.rank == r.k
    for name, h84 in (("hamming74", False), ("hamming84", True)):
        a = reports[name].error_amplification
        s, det, mis, m1, m2 = _oracle_amplification(oracle, h84)
        assert (a.single_bit_corrections, a.double_bit_detections,
                a.double_bit_miscorrections) == (s, det, mis), name
        assert a.mean_delta_dh_single == pytest.approx(m1) and a.mean_delta_dh_double == pytest.approx(m2)
        assert a.single_correction_rate == 1.0  # every single-bit error corrected
    assert reports["hamming84"].error_amplification.miscorrection_rate == 0.0
    assert reports["hamming74"].error_amplification.double_bit_miscorrections > 0  # SEC only
    g = reports["golay2412"].error_amplification
    assert g.single_bit_corrections == 24 and g.double_bit_detections == 86  # all <= 3-bit fixed
    return reports


def test_verification_cpu_backend(oracle):
    _check("cpu", oracle)


@pytest.mark.gpu
def test_verification_hip(gpu, oracle):
    hip = _check(gpu, oracle)
    cpu = _check("cpu", oracle)
    for name in hip:
        assert hip[name].error_amplification == cpu[name].error_amplification
