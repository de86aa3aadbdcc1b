"""The per-pixel random stream (oracle/philox_ref.h) pinned by Random123 known answers.

Philox4x32-10 is the generator behind cuRAND's curandStatePhilox4_32_10_t; the reference
seeds XORWOW from clock64() (ACMMP.cu:684) so its draws are not reproducible at all,
and the rebuild fixes a seeded Philox stream instead.
"""
import numpy as np


KAT = [  # Random123 kat_vectors, philox4x32 10 rounds: ctr, key -> out
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
]


def test_philox_known_answers(oracle_mod):
    for ctr, key, want in KAT:
        assert oracle_mod.philox(ctr, key).tolist() == want


def test_uniform_mapping_is_curand_uniform(oracle_mod):
    # draw n of subsequence s = word n%4 of philox({n/4, 0, s_lo, s_hi}, seed), mapped x*2^-32 + 2^-33
    seed, sub = 0x1234_5678_9ABC_DEF0, 977
    key = [seed & 0xFFFFFFFF, seed >> 32]
    for n in range(10):
        word = int(oracle_mod.philox([n // 4, 0, sub, 0], key)[n % 4])
        want = np.float32(np.float32(word) * np.float32(2.0 ** -32) + np.float32(2.0 ** -33))
        assert oracle_mod.uniform_draw(seed, sub, n) == want


def test_uniform_range_and_moments(oracle_mod):
    u = np.array([oracle_mod.uniform_draw(7, s, n) for s in range(40) for n in range(50)], np.float32)
    assert (u > 0).all() and (u <= 1).all()
    assert abs(u.mean() - 0.5) < 0.03 and abs(u.var() - 1 / 12) < 0.01
