"""Pin the oracle's RNG (test infrastructure) before trusting it.

The reference has no tests or golden vectors.  The pieces of
third-party arithmetic the render path depends on are pinned here instead:
  * the ChaCha block function against RFC 7539 §2.3.2 and OpenSSL's ChaCha20
    (libcrypto, 20 rounds; the DJB 64-bit counter/nonce layout maps onto
    OpenSSL's 16-byte IV as ctr_lo|ctr_hi|nonce_lo|nonce_hi),
  * 8 rounds against the published zero-key ChaCha8 keystream,
  * rand_core 0.9.3 seed_from_u64 (PCG32 expansion) and rand_chacha 0.9.0's
    BlockRng u64 assembly, against an independent pure-Python model.
"""
import ctypes
import ctypes.util
import struct
import subprocess

import pytest

from helpers import ORACLE_BIN, ensure_oracle

MASK = 0xFFFFFFFF


def _rotl(x, n):
    return ((x << n) | (x >> (32 - n))) & MASK


def py_chacha_block(rounds, key_words, ctr, nonce):
    s = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574, *key_words, ctr & MASK, ctr >> 32, nonce & MASK, nonce >> 32]
    x = list(s)

    def qr(a, b, c, d):
        x[a] = (x[a] + x[b]) & MASK; x[d] = _rotl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & MASK; x[b] = _rotl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & MASK; x[d] = _rotl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & MASK; x[b] = _rotl(x[b] ^ x[c], 7)

    for _ in range(rounds // 2):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return [(a + b) & MASK for a, b in zip(x, s)]


def pcg32_key(seed):
    out = []
    for _ in range(8):
        seed = (seed * 6364136223846793005 + 11634580027462260723) & ((1 << 64) - 1)
        xs = (((seed >> 18) ^ seed) >> 27) & MASK
        rot = seed >> 59
        out.append(((xs >> rot) | (xs << ((32 - rot) & 31))) & MASK)
    return out


def oracle_chacha(rounds, key_bytes, ctr, nonce, nwords):
    ensure_oracle()
    r = subprocess.run([ORACLE_BIN, "chacha", str(rounds), key_bytes.hex(), str(ctr), str(nonce), str(nwords)],
                       check=True, capture_output=True, text=True)
    return [int(w, 16) for w in r.stdout.split()]


def test_rfc7539_block_vector():
    key = bytes(range(32))
    # RFC 7539 2.3.2: counter = 1, nonce = 00000009 0000004a 00000000 (96-bit layout)
    # In the 64/64 layout: word12 = 1, word13 = 0x09000000, word14 = 0x4a000000, word15 = 0.
    ctr = 1 | (0x09000000 << 32)
    nonce = 0x4A000000
    expected = [0xE4E7F110, 0x15593BD1, 0x1FDD0F50, 0xC47120A3, 0xC7F4D1C7, 0x0368C033, 0x9AAA2204, 0x4E6CD4C3,
                0x466482D2, 0x09AA9F07, 0x05D7C214, 0xA2028BD9, 0xD19C12B5, 0xB94E16DE, 0xE883D0CB, 0x4E3C50A2]
    assert oracle_chacha(20, key, ctr, nonce, 16) == expected
    kw = list(struct.unpack("<8I", key))
    assert py_chacha_block(20, kw, ctr, nonce) == expected


def test_chacha8_zero_key_keystream():
    ks = "3e00ef2f895f40d67f5bb8e81f09a5a12c840ec3ce9a7f3b181be188ef711a1e" \
         "984ce172b9216f419f445367456d5619314a42a3da86b001387bfdb80e0cfe42"
    words = oracle_chacha(8, bytes(32), 0, 0, 16)
    assert b"".join(struct.pack("<I", w) for w in words).hex() == ks


def _openssl():
    name = ctypes.util.find_library("crypto")
    for cand in (name, "libcrypto.so.3", "libcrypto.so"):
        if not cand:
            continue
        try:
            return ctypes.CDLL(cand)
        except OSError:
            continue
    return None


@pytest.mark.parametrize("ctr,nonce", [(0, 0), (5, 123456789), (0x1234, 0xFFFFFFFF00000001)])
def test_chacha20_against_openssl(ctr, nonce):
    lib = _openssl()
    if lib is None or not hasattr(lib, "EVP_chacha20"):
        pytest.skip("libcrypto with EVP_chacha20 not available")
    lib.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
    lib.EVP_chacha20.restype = ctypes.c_void_p
    lib.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p,
                                       ctypes.c_char_p]
    lib.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                                      ctypes.c_char_p, ctypes.c_int]
    lib.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
    key = bytes((7 * i + 3) & 0xFF for i in range(32))
    iv = struct.pack("<IIII", ctr & MASK, ctr >> 32, nonce & MASK, nonce >> 32)
    ctx = lib.EVP_CIPHER_CTX_new()
    assert lib.EVP_EncryptInit_ex(ctx, lib.EVP_chacha20(), None, key, iv) == 1
    n = 64 * 3
    out = ctypes.create_string_buffer(n)
    outl = ctypes.c_int(0)
    assert lib.EVP_EncryptUpdate(ctx, out, ctypes.byref(outl), bytes(n), n) == 1
    lib.EVP_CIPHER_CTX_free(ctx)
    words = list(struct.unpack("<48I", out.raw[:n]))
    assert oracle_chacha(20, key, ctr, nonce, 48) == words


def test_seed_from_u64_zero_key():
    assert pcg32_key(0) == [0xF973F2EC, 0x45CDB581, 0x7346F087, 0xAD6CAD06, 0xE3A3D0D0, 0x67E71733, 0x72EA9BF2,
                            0xFE7D8AD7]


def py_stream(stream, count):
    """rand_chacha BlockRng<ChaCha8Core>: 4 blocks per refill, u64 = lo | hi << 32."""
    key = pcg32_key(0)
    words, blk = [], 0
    while len(words) < 2 * count:
        for b in range(4):
            words += py_chacha_block(8, key, blk + b, stream)
        blk += 4
    return [words[2 * i] | (words[2 * i + 1] << 32) for i in range(count)]


@pytest.mark.parametrize("stream", [0, 1, 4095, 1048575])
def test_pixel_stream(stream):
    ensure_oracle()
    r = subprocess.run([ORACLE_BIN, "rng", str(stream), "80"], check=True, capture_output=True, text=True)
    got = [int(x, 16) for x in r.stdout.split()]
    assert got == py_stream(stream, 80)


def py_philox2x32_10(c0, c1, key=0):
    """Philox2x32-10 (Salmon et al., SC'11; Random123 philox.h): the f32 render loop's RNG
    (kernel.hpp philox2x32_10, key 0).  Round: (hi, lo) = 0xD256D193 * c0,
    (c0, c1) = (hi ^ key ^ c1, lo); key += 0x9E3779B9 between rounds."""
    for _ in range(10):
        p = 0xD256D193 * c0
        c0, c1 = (p >> 32) ^ key ^ c1, p & 0xFFFFFFFF
        key = (key + 0x9E3779B9) & 0xFFFFFFFF
    return c0, c1


@pytest.mark.parametrize("ctr,key,want", [
    ((0x00000000, 0x00000000), 0x00000000, (0xff1dae59, 0x6cd10df2)),
    ((0xffffffff, 0xffffffff), 0xffffffff, (0x2c3f628b, 0xab4fd7ad)),
    ((0x243f6a88, 0x85a308d3), 0x13198a2e, (0xdd7ce038, 0xf62a4c12)),
])
def test_philox2x32_random123_kat(ctr, key, want):
    # Random123 kat_vectors, philox2x32 10 rounds
    assert py_philox2x32_10(*ctr, key) == want
