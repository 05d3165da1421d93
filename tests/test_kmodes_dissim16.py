"""CPU check of the <= 16-modality K-Modes dissimilarity used by kmb_assign16 (tiler_amd/csrc/kmodes.hip).

The kernel evaluates the asm dissimilarity (kmodes.pas:341-412, restated as oracle or_km_dissim and pinned by the
reference's own asm in test_oracle_kats) on a prepared 32-word row: bytes 16..79, the 4 bit planes of the 80 bytes,
and packed (byte 0 | byte 8 << 8), (byte 1 | byte 9 << 8) words.  This test restates that preparation and the
arithmetic word for word in numpy (the same bit gathering by multiplication) and compares with the oracle on rows
whose bytes are < 16, the only rows the kernel is used on (the host falls back to kmb_assign otherwise).
"""
import numpy as np
import pytest

pyoracle = pytest.importorskip("pyoracle")

M32 = 0xFFFFFFFF


def prep(row):
    d = np.frombuffer(np.ascontiguousarray(row, np.uint8).tobytes(), dtype="<u4").astype(np.uint64)
    out = [int(d[4 + w]) for w in range(16)]
    for w in range(16, 28):
        p, k = (w - 16) // 3, (w - 16) % 3
        r = 0
        for j in range(8):
            if 8 * k + j >= 20:
                break
            v = (int(d[8 * k + j]) >> p) & 0x01010101
            r |= (((v * 0x01020408) & M32) >> 24) << (4 * j)
        out.append(r & M32)
    out.append((int(d[0]) & 0xFF) | ((int(d[2]) & 0xFF) << 8))
    out.append(((int(d[0]) >> 8) & 0xFF) | (((int(d[2]) >> 8) & 0xFF) << 8))
    out += [0, 0]
    return out


def sad_u8(a, b, acc):
    return acc + sum(abs(((a >> (8 * i)) & 0xFF) - ((b >> (8 * i)) & 0xFF)) for i in range(4))


def dissim16(r, x):
    l1 = 0
    for w in range(16):
        l1 = sad_u8(r[w], x[w], l1)
    l1 = sad_u8(r[28], x[28], l1)
    hi = sad_u8(r[29], x[29], 0)
    mism = 0
    for k in range(3):
        m = (r[16 + k] ^ x[16 + k]) | (r[19 + k] ^ x[19 + k]) | (r[22 + k] ^ x[22 + k]) | (r[25 + k] ^ x[25 + k])
        mism += bin(m).count("1")
    return (mism << 11) + l1 + (hi << 8)


def kmodes_rows(rng, n):
    rows = np.zeros((n, 80), np.uint8)
    rows[:, :64] = rng.integers(0, 16, (n, 64))
    rows[:, 64:] = rng.integers(0, 2, (n, 16))  # zone flags (main.pas:4142-4164)
    return rows


def test_dissim16_matches_asm_restatement():
    rng = np.random.default_rng(7)
    rows = kmodes_rows(rng, 300)
    items = kmodes_rows(rng, 300)
    items[:50] = rows[:50]                       # identical rows: 0
    items[50:60, :64] = 15 - rows[50:60, :64]    # every palette byte differs
    full = rng.integers(0, 16, (40, 80)).astype(np.uint8)  # any byte value < 16 in every position
    rows = np.concatenate([rows, full])
    items = np.concatenate([items, rng.integers(0, 16, (40, 80)).astype(np.uint8)])
    for r, x in zip(rows, items):
        assert dissim16(prep(r), prep(x)) == pyoracle.km_dissim(r, x)


def test_dissim16_extremes():
    z = np.zeros(80, np.uint8)
    f = np.full(80, 15, np.uint8)
    for r, x in ((z, f), (f, z), (z, z), (f, f)):
        assert dissim16(prep(r), prep(x)) == pyoracle.km_dissim(r, x)
    # a single differing byte at every position, both directions
    for k in range(80):
        a = z.copy()
        a[k] = 15
        assert dissim16(prep(a), prep(z)) == pyoracle.km_dissim(a, z)
        assert dissim16(prep(z), prep(a)) == pyoracle.km_dissim(z, a)
