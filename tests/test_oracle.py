"""Pin the CPU oracle against the reference's golden vectors (CPU-only).

The fixtures in tests/golden/ were produced by tools/gen_golden.py running the
reference's own Triton kernels under TRITON_INTERPRET=1.  If these pass, the
oracle is a trustworthy checker for the HIP kernels.
"""

import hashlib

import numpy as np
import pytest

GOLAY_TABLE_SHA256 = "e60694b90298cb14647b39f3fb1e2e6af485503d333ca85b68eda0e24ba565ca"


def test_golden_manifest_hashes(manifest):
    import os
    from tests.conftest import GOLDEN
    for name, entry in manifest.items():
        if name.startswith("_"):
            continue
        with open(os.path.join(GOLDEN, entry["file"]), "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == entry["sha256"], name


def test_hamming_all_bytes(oracle, golden):
    g = golden("hamming")
    x = g["inputs"]
    assert np.array_equal(oracle.hamming74_encode(x), g["enc74"])
    assert np.array_equal(oracle.hamming84_encode(x), g["enc84"])
    d, f, st = oracle.hamming74_decode(x)
    assert np.array_equal(d, g["dec74_data"]) and np.array_equal(f, g["dec74_flag"])
    assert st == tuple(g["dec74_stats"].tolist())
    d, t, st = oracle.hamming84_decode(x)
    assert np.array_equal(d, g["dec84_data"]) and np.array_equal(t, g["dec84_type"])
    assert st == tuple(g["dec84_stats"].tolist())
    # 112 corrected / 112 detected over all 256 bytes
    assert st == (112, 112)


def test_golay_tables(oracle, golden):
    g = golden("golay")
    table = oracle.golay_syndrome_table()
    assert np.array_equal(table, g["table"])
    assert hashlib.sha256(table.astype("<i4").tobytes()).hexdigest() == GOLAY_TABLE_SHA256
    assert (table >= 0).sum() == 2325 and (table == -1).sum() == 1771
    assert np.array_equal(oracle.golay_h_row_masks().astype(np.int64), g["h_row_masks"])


def test_golay_encode_decode(oracle, golden):
    g = golden("golay")
    assert np.array_equal(oracle.golay_encode(g["enc_in"]), g["enc_out"])
    trip, cnt, st = oracle.golay_decode(g["dec_in"])
    assert np.array_equal(trip, g["dec_trip"])
    assert np.array_equal(cnt, g["dec_count"])
    assert st == tuple(g["dec_stats"].tolist())
    # every codeword with <=3 injected errors is corrected back to its data
    nerr = g["dec_nerr"]
    ok = nerr <= 3
    assert np.array_equal(cnt[: nerr.size][ok], nerr[ok].astype(np.uint8))


def test_golay_linear_parity_identity(oracle):
    """syndrome(cw) == (cw>>12) ^ P(cw & 0xFFF): the identity the HIP decode uses."""
    d = np.arange(4096)
    trip = np.stack([d & 15, (d >> 4) & 15, (d >> 8) & 15], 1).astype(np.uint8)
    parity = (oracle.golay_encode(trip).astype(np.int64) >> 12) & 0xFFF
    h = oracle.golay_h_row_masks().astype(np.int64)
    rng = np.random.default_rng(0)
    w = rng.integers(0, 2**24, size=20000)
    syn = np.zeros_like(w)
    for i in range(12):
        x = w & h[i]
        par = np.zeros_like(x)
        for b in range(24):
            par ^= (x >> b) & 1
        syn |= par << i
    assert np.array_equal(syn, ((w >> 12) & 0xFFF) ^ parity[w & 0xFFF])


@pytest.mark.parametrize("tag", ["inject", "inject_vec"])
def test_inject_golden(oracle, golden, manifest, tag):
    g = golden(tag)
    cases = manifest[tag]["params"]["cases"]
    for i, c in enumerate(cases):
        x = g[f"c{i}_in"]
        if tag == "inject":
            out, cnt, st = oracle.inject(x, c["ber"], c["n_bits"], c["seed"])
        else:
            out, cnt, st = oracle.inject_vectorized(x, c["ber"], c["n_bits"], c["seed"])
        assert np.array_equal(out, g[f"c{i}_out"]), (tag, c)
        assert st == tuple(g[f"c{i}_stats"].tolist()), (tag, c)
        # per-element counts are the popcount of the flip mask
        diff = (x.astype(np.int64) ^ out.astype(np.int64)) & 0xFFFFFFFF
        pc = np.array([bin(v).count("1") for v in diff], dtype=np.uint8)
        assert np.array_equal(cnt, pc)


def test_inject_sharding_matches_flat(oracle):
    """A shard with (global_n, offset0) reproduces the flat run bit-for-bit."""
    rng = np.random.default_rng(3)
    x = rng.integers(0, 2**24, size=3000).astype(np.int32)
    full, _, _ = oracle.inject(x, 0.05, 24, seed=42)
    parts = [oracle.inject(x[a:b], 0.05, 24, seed=42, global_n=3000, offset0=a)[0]
             for a, b in ((0, 1000), (1000, 2500), (2500, 3000))]
    assert np.array_equal(np.concatenate(parts), full)


def test_philox_known_answer(oracle):
    # Random123 Philox4x32-10 known-answer vectors (counter, key) -> output
    assert list(oracle.philox(0, 0, 0, 0, 0, 0)) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C,
                                                      0x9B00DBD8]
    assert list(oracle.philox(0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF,
                              0xFFFFFFFF, 0xFFFFFFFF)) == [0x408F276D, 0x41C83B0E,
                                                           0xA20BC7C6, 0x6D5451FD]


def test_interp_golden(oracle, golden, manifest):
    g = golden("interp")
    for i, c in enumerate(manifest["interp"]["params"]["cases"]):
        out = oracle.interpolate_double_errors(g[f"c{i}_q"], g[f"c{i}_err"], seq_dim=c["seq_dim"])
        assert np.array_equal(out, g[f"c{i}_out"]), c


def test_quantize_and_fused_golden(oracle, golden, manifest):
    g = golden("fused")
    for i, c in enumerate(manifest["fused"]["params"]["cases"]):
        q, s = oracle.quantize_rows(g[f"c{i}_x"])
        assert np.array_equal(q, g[f"c{i}_torch_q"]), c
        assert np.array_equal(s, g[f"c{i}_torch_scale"]), c
        assert np.array_equal(oracle.hamming84_encode(q), g[f"c{i}_cw84"])
        assert np.array_equal(oracle.hamming74_encode(q), g[f"c{i}_cw74"])
        dq, nc = oracle.decode_dequant_h84(g[f"c{i}_cw_noisy"], g[f"c{i}_s84"])
        assert np.array_equal(dq, g[f"c{i}_dq"]), c
        assert nc == int(g[f"c{i}_ncorr"][0])
