"""Perlin textures (Noise / Marble, lib/textures/noise.rs, marble.rs): CPU checks.

The arithmetic comes from third-party crates absent from /root/reference (noise
0.9.0, rand 0.8.5, rand_xorshift 0.3.0; Cargo.lock).  Pinned here:
  * rand_xorshift's XorShiftRng against the crate's own published test vectors
    (`test_xorshift_true_values`, `test_xorshift_construction`);
  * the permutation-table shuffle: product (libnrt.so) == oracle == an
    independent Python model of rand 0.8.5's `shuffle` / `gen_range`;
  * size-independent properties of noise 0.9's perlin_3d / Fbm (zero on the
    integer lattice, |Fbm| bound, marble in [0, 1]).
The perlin_3d / Fbm arithmetic itself has no reference vector: parity with the
reference is unpinned beyond the restatement.
"""
import math
import subprocess

import numpy as np
import pytest

import nrt
from helpers import ORACLE_BIN, ensure_oracle

M32 = 0xFFFFFFFF


def oracle(*args):
    ensure_oracle()
    return subprocess.run([ORACLE_BIN, *map(str, args)], check=True, capture_output=True, text=True).stdout.split()


def py_xorshift(seed16):
    x, y, z, w = (int.from_bytes(bytes(seed16[4 * i:4 * i + 4]), "little") for i in range(4))
    while True:
        t = (x ^ (x << 11)) & M32
        x, y, z = y, z, w
        w = (w ^ (w >> 19) ^ (t ^ (t >> 8))) & M32
        yield w


def py_permutation(seed):
    # PermutationTable::new: seed bytes [1,0,0,0, s x3]; rand 0.8.5 shuffle with gen_range(0..i+1)
    real = [1, 0, 0, 0] + list(seed.to_bytes(4, "little")) * 3
    rng = py_xorshift(real)
    v = list(range(256))
    for i in range(255, 0, -1):
        rng_range = i + 1
        zone = ((rng_range << (32 - rng_range.bit_length())) & M32) - 1
        while True:
            m = next(rng) * rng_range
            if (m & M32) <= zone:
                j = m >> 32
                break
        v[i], v[j] = v[j], v[i]
    return v


def test_xorshift_published_vectors():
    # rand_xorshift 0.3.0 src/lib.rs test_xorshift_true_values
    got = [int(v) for v in oracle("xorshift", bytes(range(16, 0, -1)).hex(), 9)]
    assert got == [2081028795, 620940381, 269070770, 16943764, 854422573, 29242889, 1550291885, 1227154591,
                   271695242]
    # test_xorshift_construction: from_seed([1..=16]).next_u64() (next_u64 = lo | hi << 32)
    lo, hi = (int(v) for v in oracle("xorshift", bytes(range(1, 17)).hex(), 2))
    assert lo | hi << 32 == 4325440999699518727
    assert list(np.array(got)) == [v for v, _ in zip(py_xorshift(list(range(16, 0, -1))), range(9))]


@pytest.mark.parametrize("seed", [0, 1, 2, 7, 12345, 0xFFFFFFFF])
def test_permutation_tables_agree(seed):
    want = py_permutation(seed)
    assert sorted(want) == list(range(256))
    assert [int(v) for v in oracle("perm", seed)] == want
    assert nrt.debug_perlin_permutation(seed).tolist() == want


def test_perlin_zero_on_lattice():
    # perlin_3d at integer points: distance = 0 -> every k term vanishes but k0 = g000 = 0
    for p in [(0, 0, 0), (1, 2, 3), (-4, 7, -2), (100, -33, 5)]:
        assert float.fromhex(oracle("noise", 0, 1, 1.0, 2.0, 0.5, *p)[0]) == 0.0


def test_noise_bound_and_marble_range():
    rng = np.random.default_rng(5)
    pts = rng.uniform(-40, 40, size=(40, 3))
    for oct_, pers in [(1, 0.5), (8, 0.5), (4, 0.8)]:
        scale = 1.0 / sum(pers ** k for k in range(1, oct_ + 1))
        bound = scale * sum(pers ** k for k in range(oct_))
        vals = [float.fromhex(oracle("noise", 3, oct_, 0.2, 2 * math.pi / 3, pers, *p)[0]) for p in pts[:10]]
        assert all(0.0 <= v <= bound for v in vals)
        assert any(v > 0 for v in vals)
    m = [float.fromhex(oracle("marble", 0, 0.2, *p)[0]) for p in pts]
    assert all(0.0 <= v <= 1.0 for v in m)
    assert max(m) - min(m) > 0.2  # actually varies
