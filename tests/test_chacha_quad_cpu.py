"""The four-lane ChaCha20 schedule of chacha20_block_quad (fhe-icp_amd/csrc/
prng.h: lane q holds state column q; the diagonal round runs after rotating
rows 1-3 by 1, 2, 3 lanes, DPP quad_perm 0x39 / 0x4e / 0x93, and back)
restated on four emulated lanes and checked against the oracle's RFC 8439
block (oracle/tfhe_ref.c ref_chacha20_block), and the even/odd-lane u64 word
assembly k_encrypt_linear does from it (quad_perm 0xb1). The device code
itself is checked bit for bit on the GPU (test_encrypt_linear_fused_bit_exact)."""
import numpy as np
import pytest

M32 = 0xFFFFFFFF


def _rotl(x, b):
    return ((x << b) | (x >> (32 - b))) & M32


def _qr(a, b, c, d):
    a = (a + b) & M32; d = _rotl(d ^ a, 16)
    c = (c + d) & M32; b = _rotl(b ^ c, 12)
    a = (a + b) & M32; d = _rotl(d ^ a, 8)
    c = (c + d) & M32; b = _rotl(b ^ c, 7)
    return a, b, c, d


def _quad_perm(vals, ctrl):
    """DPP quad_perm: lane q reads lane (ctrl >> 2q) & 3 of its quad."""
    return [vals[(ctrl >> (2 * q)) & 3] for q in range(4)]


def chacha_quad(key, counter, tag, ident):
    const = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574]
    a = list(const)
    b = [int(key[q]) for q in range(4)]
    c = [int(key[4 + q]) for q in range(4)]
    d = [counter, tag, ident & M32, ident >> 32]
    a0, b0, c0, d0 = list(a), list(b), list(c), list(d)
    for _ in range(10):
        a, b, c, d = map(list, zip(*[_qr(a[q], b[q], c[q], d[q]) for q in range(4)]))
        b, c, d = _quad_perm(b, 0x39), _quad_perm(c, 0x4E), _quad_perm(d, 0x93)
        a, b, c, d = map(list, zip(*[_qr(a[q], b[q], c[q], d[q]) for q in range(4)]))
        b, c, d = _quad_perm(b, 0x93), _quad_perm(c, 0x4E), _quad_perm(d, 0x39)
    # lane q: out[r] = word q + 4 r
    return [[(x + y) & M32 for x, y in zip(row, row0)] for row, row0 in ((a, a0), (b, b0), (c, c0), (d, d0))]


@pytest.mark.parametrize("counter,tag,ident", [(0, 8, 77), (5, 8, (3 << 40) + 12345), (127, 7, 2 ** 63 + 9)])
def test_quad_schedule_matches_rfc8439(oracle_lib, counter, tag, ident):
    from oracle import tfhe_ref as ref
    key = ref.key_from_seed(8)
    want = ref.chacha20_block(key, counter, np.array([tag, ident & M32, ident >> 32], np.uint32))
    rows = chacha_quad(key, counter, tag, ident)
    got = [rows[r][q] for r in range(4) for q in range(4)]  # word q + 4 r
    got_by_index = [0] * 16
    for r in range(4):
        for q in range(4):
            got_by_index[q + 4 * r] = rows[r][q]
    assert got_by_index == [int(v) for v in want]
    assert sorted(got) == sorted(int(v) for v in want)
    # the u64 words k_encrypt_linear assembles: even lane q, row r holds the
    # low half of word j = (q + 4 r) / 2, its odd neighbour (quad_perm 0xb1)
    # the high half
    words = {}
    for r in range(4):
        hi = _quad_perm(rows[r], 0xB1)
        for q in (0, 2):
            words[(q + 4 * r) >> 1] = rows[r][q] | (hi[q] << 32)
    assert [words[j] for j in range(8)] == [int(want[2 * j]) | (int(want[2 * j + 1]) << 32) for j in range(8)]
