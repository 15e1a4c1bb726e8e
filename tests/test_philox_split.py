"""The tail session's Philox split (pbn_kernels.hip, k_env tail mode, the draw lambda): the 64 calls of a
block differ in counter word 0 only (words 1-3 are the session's call index and env id), so half of
rounds 0 and 1 is computed once per session and a call does 18 multiplies instead of 20. Restated
here in Python integers and checked against the oracle's Philox4x32-10 (Random123 KAT-checked in
test_oracle.py), word for word, on random keys, counters and env ids (CPU only)."""
import numpy as np

M0, M1, W0, W1, M32 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85, 0xFFFFFFFF
STREAM_ENV = 3


def session(seed, c1, gid):
    """The per-session scalars of the split (names as in the kernel)."""
    sk0, sk1 = seed & M32, seed >> 32
    g2, g3 = gid & M32, ((gid >> 32) & 0xFFFFFF) | (STREAM_ENV << 24)
    p1u = M1 * g2
    a0 = (p1u >> 32) ^ c1 ^ sk0
    u0 = g3 ^ sk1
    v1 = (p1u & M32) ^ ((sk0 + W0) & M32)
    p0u = M0 * a0
    h1 = (p0u >> 32) ^ ((sk1 + W1) & M32)
    l1 = p0u & M32
    return sk0, sk1, u0, v1, h1, l1


def draw_split(s, c0):
    sk0, sk1, u0, v1, h1, l1 = s
    p0 = M0 * c0  # round 0: the lane's half
    y = (p0 >> 32) ^ u0
    p1 = M1 * y  # round 1: the lane's half
    w = [(p1 >> 32) ^ v1, p1 & M32, (p0 & M32) ^ h1, l1]
    k0, k1 = (sk0 + W0) & M32, (sk1 + W1) & M32
    for _ in range(2, 10):
        k0, k1 = (k0 + W0) & M32, (k1 + W1) & M32
        q0, q1 = M0 * w[0], M1 * w[2]
        w = [(q1 >> 32) ^ w[1] ^ k0, q1 & M32, (q0 >> 32) ^ w[3] ^ k1, q0 & M32]
    return w


def test_tail_philox_split_matches_oracle(oracle_mod):
    rng = np.random.default_rng(11)
    for _ in range(60):
        seed = int(rng.integers(0, 2**63)) * 2 + int(rng.integers(0, 2))
        c1 = int(rng.integers(0, 2**32))
        gid = int(rng.integers(0, 2**40))
        s = session(seed, c1, gid)
        for c0 in [0, M32] + [int(x) for x in rng.integers(0, 2**32, size=8)]:
            ctr = [c0, c1, gid & M32, ((gid >> 32) & 0xFFFFFF) | (STREAM_ENV << 24)]
            assert draw_split(s, c0) == oracle_mod.philox4x32_10(ctr, [seed & M32, seed >> 32])
