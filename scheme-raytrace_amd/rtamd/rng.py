"""Counter-based random numbers (Philox4x32-10) shared by the host, the GPU
kernels and the oracle.

The reference draws every random number from one global srfi-27 stream
(`random-real`, 37 call sites), so the number of draws per pixel depends on
the data and a parallel GPU cannot replay it.  The drop-in replaces it by
counter-based streams:

* path stream (GPU kernels + oracle): key = seed, counter =
  (draw >> 1, sample, pixel, 0); draw d uses words (0,1) if d is even else
  (2,3) of the Philox block.
* host stream (scene construction, Perlin tables — the reference's load-time
  draws, perlin.scm:32-36, main.scm:45-70): key = seed, counter =
  (draw >> 1, 0, 0xFFFFFFFF, 1).

A pair of 32-bit words (hi, lo) becomes u = (2k+1) * 2^-53 with
k = (hi >> 12) << 32 | lo: 52 random bits, always inside (0, 1) like
srfi-27's random-real.
"""

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    c0, c1, c2, c3 = ctr
    k0, k1 = key
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


def u32pair_unit(hi, lo):
    k = ((hi >> 12) << 32) | lo
    return (2 * k + 1) * (1.0 / 9007199254740992.0)


def split_seed(seed):
    seed &= (1 << 64) - 1
    return (seed & MASK, seed >> 32)


def path_draw(seed, pix, smp, d):
    """Draw number d of the path stream (seed, pixel, sample)."""
    w = philox4x32_10((d >> 1, smp & MASK, pix & MASK, 0), split_seed(seed))
    return u32pair_unit(w[2], w[3]) if d & 1 else u32pair_unit(w[0], w[1])


class HostStream:
    """Sequential host-side replacement of the global `random-real`."""

    def __init__(self, seed):
        self.key = split_seed(seed)
        self.count = 0
        self._blk = None
        self._w = None

    def random_real(self):
        d = self.count
        self.count += 1
        b = d >> 1
        if b != self._blk:
            self._w = philox4x32_10((b & MASK, 0, MASK, 1), self.key)
            self._blk = b
        w = self._w
        return u32pair_unit(w[2], w[3]) if d & 1 else u32pair_unit(w[0], w[1])

    __call__ = random_real
