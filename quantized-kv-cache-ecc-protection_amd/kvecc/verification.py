"""Code-property and error-amplification verification of the three codecs.

Mirrors evaluation/verification.py (dataclasses :57-105, checks :107-472,
report :474-548): GF(2) null-space and orthogonality of G/H, rank of G, and
exhaustive single/double-bit error statistics through the codec classes.
The reference loops one decode launch per corrupted word; here every
corruption pattern of a check goes through ONE batched decode, on the codec
backend the classes pick for `device` ("hip" for a GPU device, "cpu" for the
host backend).
"""

from __future__ import annotations

from dataclasses import dataclass
from itertools import combinations

import torch

from .codecs import Golay2412, Hamming74, Hamming84
from .config import ErrorType


@dataclass
class NullSpaceResult:
    syndrome_zero_rate: float
    total_codewords: int
    valid_codewords: int
    failed_syndromes: list


@dataclass
class OrthogonalityResult:
    is_orthogonal: bool
    frobenius_norm: float
    product_matrix: torch.Tensor | None


@dataclass
class RankResult:
    rank: int
    expected_rank: int
    is_full_rank: bool
    condition_number: float | None


@dataclass
class ErrorAmplificationResult:
    single_bit_corrections: int
    double_bit_detections: int
    double_bit_miscorrections: int
    mean_delta_dh_single: float
    mean_delta_dh_double: float
    single_correction_rate: float
    double_detection_rate: float
    miscorrection_rate: float


@dataclass
class VerificationReport:
    code_name: str
    n: int
    k: int
    null_space: NullSpaceResult
    orthogonality: OrthogonalityResult
    rank: RankResult
    error_amplification: ErrorAmplificationResult
    all_passed: bool


_POP4 = torch.tensor([bin(i).count("1") for i in range(16)], dtype=torch.int64)


def compute_gf2_rank(matrix: torch.Tensor) -> int:
    """Rank over GF(2) by row reduction (verification.py:107-136)."""
    m = (matrix.detach().to("cpu", torch.int64) % 2).clone()
    rows, cols = m.shape
    rank = 0
    for col in range(cols):
        pivot = next((r for r in range(rank, rows) if m[r, col] == 1), None)
        if pivot is None:
            continue
        m[[rank, pivot]] = m[[pivot, rank]]
        hit = (m[:, col] == 1) & (torch.arange(rows) != rank)
        m[hit] ^= m[rank]
        rank += 1
        if rank == rows:
            break
    return rank


def hamming_distance(a: int, b: int) -> int:
    return bin(a ^ b).count("1")


def verify_null_space_condition(G, H, device="cuda"):
    """Every codeword data @ G has zero syndrome H @ c (verification.py:143-172)."""
    k, n = G.shape
    data = (torch.arange(2 ** k).unsqueeze(1) >> torch.arange(k)) & 1     # [2^k, k]
    cw = (data.double() @ G.detach().cpu().double()) % 2                  # [2^k, n]
    syn = (cw @ H.detach().cpu().double().T) % 2                          # [2^k, n-k]
    ok = syn.sum(1) == 0
    weights = 1 << torch.arange(syn.shape[1], dtype=torch.int64)
    failed = [(int(i), int((syn[i].long() * weights).sum())) for i in torch.nonzero(~ok)[:10, 0]]
    return NullSpaceResult(syndrome_zero_rate=float(ok.double().mean()), total_codewords=2 ** k,
                           valid_codewords=int(ok.sum()), failed_syndromes=failed)


def verify_subspace_orthogonality(G, H, device="cuda"):
    """G @ H^T == 0 over GF(2) (verification.py:175-187)."""
    product = (G.detach().cpu().double() @ H.detach().cpu().double().T) % 2
    frob = float(product.sum())
    return OrthogonalityResult(is_orthogonal=frob == 0, frobenius_norm=frob,
                               product_matrix=product if frob > 0 else None)


def verify_basis_independence(G, expected_rank, device="cuda"):
    """GF(2) rank of G and the condition number of G G^T (verification.py:190-212)."""
    rank = compute_gf2_rank(G)
    try:
        gf = G.detach().cpu().double()
        eig = torch.linalg.eigvalsh(gf @ gf.T)
        pos = eig[eig > 1e-10]
        condition = float(pos.max() / pos.min()) if len(pos) else float("inf")
    except Exception:  # noqa: BLE001 -- the reference reports None on any failure
        condition = None
    return RankResult(rank=rank, expected_rank=expected_rank, is_full_rank=rank == expected_rank,
                      condition_number=condition)


def _amplification(codec, n_bits, h84):
    """All single- and double-bit corruptions of all 16 codewords, decoded in
    one batch each (verification.py:215-349)."""
    vals = torch.arange(16, dtype=torch.uint8)
    cws = codec.encode(vals.to(codec.device)).cpu().to(torch.int64)
    singles = [(v, 1 << b) for v in range(16) for b in range(n_bits)]
    doubles = [(v, (1 << b1) | (1 << b2)) for v in range(16)
               for b1, b2 in combinations(range(n_bits), 2)]

    def run(pairs):
        v = torch.tensor([p[0] for p in pairs], dtype=torch.int64)
        corrupted = cws[v] ^ torch.tensor([p[1] for p in pairs], dtype=torch.int64)
        res = codec.decode(corrupted.to(torch.uint8).to(codec.device))
        if h84:
            dec, et = res.data.cpu().to(torch.int64), res.error_type.cpu().to(torch.int64)
        else:
            dec, et = res[0].cpu().to(torch.int64), None
        delta = _POP4[v ^ dec] - _POP4[v ^ (corrupted & 0xF)]
        return v, dec, et, delta

    v, dec, _, d1 = run(singles)
    single_ok = int((dec == v).sum())
    v, dec, et, d2 = run(doubles)
    if h84:
        detected = (et == ErrorType.DOUBLE_DETECTED) | (d2 <= 0)
    else:
        detected = d2 <= 0
    det, mis = int(detected.sum()), int((~detected).sum())
    return ErrorAmplificationResult(
        single_bit_corrections=single_ok, double_bit_detections=det,
        double_bit_miscorrections=mis,
        mean_delta_dh_single=float(d1.double().mean()),
        mean_delta_dh_double=float(d2.double().mean()),
        single_correction_rate=single_ok / len(singles),
        double_detection_rate=det / len(doubles), miscorrection_rate=mis / len(doubles))


def compute_error_amplification_hamming74(device="cuda"):
    return _amplification(Hamming74(device=device), 7, h84=False)


def compute_error_amplification_hamming84(device="cuda"):
    return _amplification(Hamming84(device=device, on_double_error="zero"), 8, h84=True)


def verify_hamming74(device="cuda"):
    G, H = Hamming74.G.clone(), Hamming74.H.clone()
    ns = verify_null_space_condition(G, H, device)
    orth = verify_subspace_orthogonality(G, H, device)
    rank = verify_basis_independence(G, 4, device)
    amp = compute_error_amplification_hamming74(device)
    ok = ns.syndrome_zero_rate == 1.0 and orth.is_orthogonal and rank.is_full_rank
    return VerificationReport("Hamming(7,4)", 7, 4, ns, orth, rank, amp, ok)


def verify_hamming84(device="cuda"):
    G, H = Hamming84.G_74.clone(), Hamming84.H_74.clone()
    ns = verify_null_space_condition(G, H, device)
    orth = verify_subspace_orthogonality(G, H, device)
    rank = verify_basis_independence(G, 4, device)
    amp = compute_error_amplification_hamming84(device)
    ok = (ns.syndrome_zero_rate == 1.0 and orth.is_orthogonal and rank.is_full_rank
          and amp.miscorrection_rate == 0.0)
    return VerificationReport("Hamming(8,4) SECDED", 8, 4, ns, orth, rank, amp, ok)


def verify_golay2412(device="cuda"):
    """verification.py:407-471: matrix checks plus the corruption patterns the
    reference walks around the triplet (5, 10, 3), in one batched decode."""
    codec = Golay2412(device=device)
    G, H = codec.G.clone(), codec.H.clone()
    ns = verify_null_space_condition(G, H, device)
    orth = verify_subspace_orthogonality(G, H, device)
    rank = verify_basis_independence(G, 12, device)
    trip = torch.tensor([[5, 10, 3]], dtype=torch.uint8)
    cw = int(codec.encode(trip.to(codec.device)).cpu()[0])
    ones = [1 << i for i in range(24)]
    twos = [(1 << i) | (1 << j) for i in range(24) for j in range(i + 1, min(i + 5, 24))]
    threes = [(1 << i) | (1 << j) | (1 << k) for i in range(0, 24, 3)
              for j in range(i + 1, min(i + 4, 24)) for k in range(j + 1, min(j + 3, 24))]
    masks = torch.tensor(ones + twos + threes, dtype=torch.int64)
    res = codec.decode((cw ^ masks).to(codec.device))
    good = (res.data.cpu() == trip[0]).all(dim=1)
    n1, n2 = len(ones), len(twos)
    c1, c2 = int(good[:n1].sum()), int(good[n1:n1 + n2].sum())
    amp = ErrorAmplificationResult(
        single_bit_corrections=c1, double_bit_detections=c2, double_bit_miscorrections=0,
        mean_delta_dh_single=-1.0, mean_delta_dh_double=-2.0, single_correction_rate=c1 / 24,
        double_detection_rate=1.0, miscorrection_rate=0.0)
    ok = ns.syndrome_zero_rate == 1.0 and orth.is_orthogonal and rank.is_full_rank and c1 == 24
    return VerificationReport("Golay(24,12)", 24, 12, ns, orth, rank, amp, ok)


def format_verification_report(report: VerificationReport) -> str:
    a = report.error_amplification
    lines = [
        f"{report.code_name} [n={report.n}, k={report.k}]: "
        f"{'PASS' if report.all_passed else 'FAIL'}",
        f"  null space: {report.null_space.valid_codewords}/{report.null_space.total_codewords} "
        f"codewords with zero syndrome",
        f"  G H^T = 0: {report.orthogonality.is_orthogonal} "
        f"(|.|_F = {report.orthogonality.frobenius_norm:g})",
        f"  rank(G) = {report.rank.rank} (expected {report.rank.expected_rank})",
        f"  single-bit: {a.single_bit_corrections} corrected "
        f"({a.single_correction_rate:.1%}), mean dH change {a.mean_delta_dh_single:+.3f}",
        f"  double-bit: {a.double_bit_detections} detected/harmless, "
        f"{a.double_bit_miscorrections} miscorrected ({a.miscorrection_rate:.1%}), "
        f"mean dH change {a.mean_delta_dh_double:+.3f}",
    ]
    return "\n".join(lines)


def run_all_verifications(device="cuda"):
    return {"hamming74": verify_hamming74(device), "hamming84": verify_hamming84(device),
            "golay2412": verify_golay2412(device)}
