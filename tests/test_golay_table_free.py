"""The table-free Golay(24,12) correction of tools/exp/golay_tf_exp.hip against
the reference's 4096-entry syndrome table (golden fixture, generated from the
reference's config.py:403-457 ordering) on every syndrome, and its decode
against the C oracle on all 2^24 received words.

B is symmetric with B B = I, so u = s B undoes the data half: the four weight
tests (wt(s) <= 3; wt(u) <= 3; wt(s ^ B_i) <= 2; wt(u ^ B_j) <= 2) find the
unique coset leader of weight <= 3, which is exactly the table's entry; every
other syndrome is the table's -1 (uncorrectable).  The GPU probe decodes a full
[8,4096,32,128] cache at BER 1e-2 and 5e-2 bit-equal to the product
(profiles/r05/golay_tf_ab*.log)."""

import numpy as np

ROWS = (0xA3B, 0xD1D, 0xE8E, 0xB47, 0xDA3, 0xED1, 0xF68, 0xBB4, 0x9DA, 0x8ED, 0xC76, 0x7FF)


def _par(x):
    p = 0
    for j in range(12):
        if x >> j & 1:
            p ^= ROWS[j]
    return p


def _wt(x):
    return bin(x).count("1")


def table_free_pattern(s):
    """24-bit error pattern (data bits 0-11, parity bits 12-23) or -1."""
    if _wt(s) <= 3:
        return s << 12
    u = _par(s)
    if _wt(u) <= 3:
        return u
    for i, r in enumerate(ROWS):
        if _wt(s ^ r) <= 2:
            return (1 << i) | (s ^ r) << 12
    for j, r in enumerate(ROWS):
        if _wt(u ^ r) <= 2:
            return (u ^ r) | (1 << j) << 12
    return -1


def test_b_is_an_involution():
    assert all(_par(_par(1 << i)) == 1 << i for i in range(12))
    assert all((ROWS[i] >> j & 1) == (ROWS[j] >> i & 1) for i in range(12) for j in range(12))


def test_table_free_equals_reference_table(golden):
    table = golden("golay")["table"].astype(np.int64)
    assert table.shape == (4096,)
    got = np.array([table_free_pattern(s) for s in range(4096)], np.int64)
    assert np.array_equal(got, table)
    assert int((got < 0).sum()) == 4096 - 2325  # coset leaders of weight <= 3: 1 + 24 + 276 + 2024


def test_table_free_decode_equals_oracle_on_every_word(oracle):
    """All 2^24 received words: data = low 12 bits XOR the table-free data
    correction, counts = the pattern's weight (4 = uncorrectable, data kept),
    against the C oracle's decode (golay_triton.py:213-295 restated)."""
    pat = np.array([table_free_pattern(s) for s in range(4096)], np.int64)
    par = np.zeros(4096, np.int64)
    for x in range(4096):
        par[x] = _par(x)
    w = np.arange(1 << 24, dtype=np.int64)
    s = ((w >> 12) ^ par[w & 0xFFF]) & 0xFFF
    e = pat[s]
    unc = e < 0
    data = np.where(unc, w & 0xFFF, (w ^ np.where(unc, 0, e)) & 0xFFF)
    wt_e = np.zeros(1 << 24, np.int64)
    ee = np.where(unc, 0, e)
    for b in range(24):
        wt_e += (ee >> b) & 1
    cnt = np.where(unc, 4, wt_e)
    trip, ocnt, _ = oracle.golay_decode(w.astype(np.int32))
    odata = trip[:, 0].astype(np.int64) | trip[:, 1].astype(np.int64) << 4 | trip[:, 2].astype(np.int64) << 8
    assert np.array_equal(odata, data)
    assert np.array_equal(ocnt.astype(np.int64), cnt)
