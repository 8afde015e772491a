"""Index algebra the multi-bit blind rotation relies on (no GPU): a pure-Python
restatement of br_v4.h's layouts (jof, rpos), mb::exponent, the level-1
source-lane product quarters of mb_rotate (mb_xpose) with the key order
k_bsk_to_fft_v4 writes for them (perm), and the two lane swaps that hand the
products to their owners (fhe-icp_amd/csrc/k_blind_rotate.h)."""
import itertools

import pytest

LAYS = [[6, 7, 8, 0, 1, 2, 3, 4, 5], [3, 4, 5, 0, 1, 2, 6, 7, 8], [0, 1, 2, 4, 5, 8, 3, 6, 7]]
LA, LB, LC = 0, 1, 2
RC = [[1, 2, 4, 7, 16], [2, 4, 8, 16, 31], [2, 4, 8, 16, 30], [0, 0, 0, 0, 0]]  # R2F, R2I, R1F, R1I
R2F, R2I, R1F, R1I = 0, 1, 2, 3
SCR = 576


def jof(li, lane, u):
    j = 0
    for b in range(3):
        j |= ((u >> b) & 1) << LAYS[li][b]
    for b in range(6):
        j |= ((lane >> b) & 1) << LAYS[li][3 + b]
    return j


def rpos(r, j):
    return j + sum(RC[r][k] * ((j >> (4 + k)) & 1) for k in range(5))


def bitrev9(j):
    return int(f"{j:09b}"[::-1], 2)


def exponent(lane, u):
    return (4 * bitrev9(jof(LC, lane, u)) + 1) & 2047


def key_pos(u, lane):
    """k_bsk_to_fft_v4 with perm: where the value of output point (slot u, lane) is stored."""
    return (2 * (lane >> 4) + (u & 1)) * 64 + 16 * (u >> 1) + (lane & 15)


def test_key_order_is_a_permutation_and_matches_the_product_reads():
    pos = {key_pos(u, lane): (u, lane) for u in range(8) for lane in range(64)}
    assert sorted(pos) == list(range(512))
    # the product wave of quarter g loads key slot 2g + t at lane l and takes
    # it as point (slot 2 (l >> 4) + t, lane 16 g + (l & 15)), whose F it reads
    for g, t, l in itertools.product(range(4), range(2), range(64)):
        assert pos[(2 * g + t) * 64 + l] == (2 * (l >> 4) + t, 16 * g + (l & 15))


def test_quarters_cover_every_point_once():
    pts = [(2 * (l >> 4) + t, 16 * g + (l & 15)) for g in range(4) for t in range(2) for l in range(64)]
    assert sorted(pts) == [(u, lane) for u in range(8) for lane in range(64)]


def test_second_slot_exponent_is_first_plus_half_turn():
    # pa ^= (a & 1) << 14 for t = 1: slot 2q + 1's exponent is slot 2q's + 1024
    for lane, q in itertools.product(range(64), range(4)):
        assert exponent(lane, 2 * q + 1) == (exponent(lane, 2 * q) + 1024) & 2047


def test_relayout_positions_are_additive_and_in_scratch():
    # R1F / R1I: the LA <-> LB exchange through the slot of the FHEICP_ABLDS A/B builds
    for r, li in ((R2F, LB), (R2I, LC), (R1F, LA), (R1I, LB)):
        for lane, u in itertools.product(range(64), range(8)):
            p = rpos(r, jof(li, lane, u))
            assert p == rpos(r, jof(li, lane, 0)) + rpos(r, jof(li, 0, u))
            assert p < SCR
        assert len({rpos(r, jof(li, lane, u)) for lane in range(64) for u in range(8)}) == 512


def _swap(regs, stride, lane_bit):
    """swap_bit<KIND, STRIDE> on a wave: for the register pair (u, u + stride)
    the lanes with lane_bit clear of the second register trade places with the
    lanes with lane_bit set of the first (v_permlane32_swap: bit 5,
    v_permlane16_swap: bit 4)."""
    m = 1 << lane_bit
    out = [list(r) for r in regs]
    for u in range(8):
        if u & stride:
            continue
        x, y = regs[u], regs[u + stride]
        for lane in range(64):
            if lane & m:
                out[u][lane] = y[lane ^ m]
            else:
                out[u + stride][lane] = x[lane ^ m]
    return out


@pytest.mark.parametrize("g", range(4))
def test_handoff_lane_swaps_give_each_lane_one_ciphertexts_slots(g):
    # o[gg][t] at lane 16 q + s: ciphertext gg, slot 2q + t, source lane 16 g + s
    regs = [[(u >> 1, 2 * (lane >> 4) + (u & 1), 16 * g + (lane & 15)) for lane in range(64)] for u in range(8)]
    regs = _swap(regs, 4, 5)
    regs = _swap(regs, 2, 4)
    for u, lane in itertools.product(range(8), range(64)):
        # lane 16 G + s now holds ciphertext G, slot u, source lane 16 g + s
        assert regs[u][lane] == (lane >> 4, u, 16 * g + (lane & 15))


def _read_groups():
    """ds_read_b128 lane groups (MI355X_MICROARCH.md §LDS): one LDS cycle each when the
    16 lanes hit 16 distinct 16-byte bank quads."""
    g = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
         [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
    return g + [[l + 32 for l in x] for x in g]


@pytest.mark.parametrize("r,src,dst", [(R2F, LB, LC), (R2I, LC, LB), (R1F, LA, LB), (R1I, LB, LA)])
def test_relayouts_are_bank_conflict_free(r, src, dst):
    """Each relayout's writes (8-lane ds_write_b128 groups in the source layout) and reads
    (16-lane ds_read_b128 groups in the target layout) touch distinct 16-byte quads mod 8 /
    mod 16 (tools/search_relayout.py's criterion)."""
    for u in range(8):
        for g0 in range(0, 64, 8):
            quads = {rpos(r, jof(src, lane, u)) % 8 for lane in range(g0, g0 + 8)}
            assert len(quads) == 8, (r, u, g0)
        for grp in _read_groups():
            quads = {rpos(r, jof(dst, lane, u)) % 16 for lane in grp}
            assert len(quads) == 16, (r, u, grp)
