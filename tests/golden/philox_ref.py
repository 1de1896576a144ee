"""Pure-Python Philox4x32-10 keyed uniform stream — TEST INFRASTRUCTURE.

The reference draws every random number from Python's global, unseeded
Mersenne Twister (`/root/reference/main.py:16`, `/root/reference/utils.py:9`),
so it is not reproducible.  To make golden vectors, the harness in
`gen_golden.py` replaces `uniform(a, b)` with a keyed counter-based draw; the
C oracle (`oracle/pt_oracle.c`) and the HIP kernel use the same stream:

    key   = (seed & 0xffffffff, seed >> 32)
    ctr   = (pixel_k, sample, bounce, slot >> 2)
    word  = Philox4x32-10(ctr, key)[slot & 3]
    u     = (word >> 8) * 2**-24                  in [0, 1), exact in f32
    uniform(a, b) = a + (b - a) * u               (random.uniform's formula)

Slot map (per pixel, per sample, per bounce):
    NEE light sample k in {0,1,2}: 4k = triangle pick (`utils.py:30`),
        4k+1 .. 4k+3 = barycentric u's (`utils.py:23`)
    12 = diffuse/specular select (`main.py:240`)
    13 = phi draw (`main.py:242`), 14 = theta draw (`main.py:243`)
    15 = Russian roulette (build extension; unused by the reference)
"""

M0 = 0xD2511F53
M1 = 0xCD9E8D57
W0 = 0x9E3779B9
W1 = 0xBB67AE85
MASK = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    c0, c1, c2, c3 = (int(x) & MASK for x in ctr)
    k0, k1 = (int(x) & MASK for x in key)
    for r in range(10):
        if r:
            k0 = (k0 + W0) & MASK
            k1 = (k1 + W1) & MASK
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> 32, p0 & MASK
        hi1, lo1 = p1 >> 32, p1 & MASK
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
    return (c0, c1, c2, c3)


def keyed_u(seed, pixel_k, sample, bounce, slot):
    seed = int(seed)
    words = philox4x32_10((pixel_k, sample, bounce, slot >> 2),
                          (seed & MASK, (seed >> 32) & MASK))
    return (words[slot & 3] >> 8) * (1.0 / 16777216.0)


def keyed_uniform(seed, pixel_k, sample, bounce, slot, a, b):
    return a + (b - a) * keyed_u(seed, pixel_k, sample, bounce, slot)
