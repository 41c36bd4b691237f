"""glibc rand() (random_r TYPE_3, the additive feedback generator) as a stream.

ORB-SLAM2's RANSAC draws DUtils::Random::RandomInt from the process-global
rand(), which is never seeded in stereo / RGB-D runs (glibc default seed 1;
SURVEY.md §8a C2).  PnPsolver.iterate takes the rand() values explicitly, so
callers that reproduce a reference run use this stream (or libc's own rand()).
"""


class GlibcRand:
    """r[i] = r[i-3] + r[i-31] (mod 2^32), output r >> 1, after the glibc seeding
    (16807 LCG over 31 words, 310 discarded outputs)."""

    def __init__(self, seed=1):
        self.seed(seed)

    def seed(self, seed):
        seed = seed & 0xFFFFFFFF
        if seed == 0:
            seed = 1
        r = [0] * 34
        r[0] = seed if seed < 0x80000000 else seed - (1 << 32)
        for i in range(1, 31):
            hi, lo = divmod(r[i - 1], 127773) if r[i - 1] >= 0 else (-((-r[i - 1]) // 127773),
                                                                      -((-r[i - 1]) % 127773))
            word = 16807 * lo - 2836 * hi
            if word < 0:
                word += 2147483647
            r[i] = word
        for i in range(31, 34):
            r[i] = r[i - 31]
        self._r = [x & 0xFFFFFFFF for x in r]
        for _ in range(310):
            self._next_word()

    def _next_word(self):
        r = self._r
        v = (r[-31] + r[-3]) & 0xFFFFFFFF
        r.append(v)
        if len(r) > 64:
            del r[:len(r) - 34]
        return v

    def rand(self):
        return self._next_word() >> 1

    def take(self, n):
        return [self.rand() for _ in range(n)]

    def peek(self, n):
        """The next n values without consuming them."""
        saved = list(self._r)
        out = self.take(n)
        self._r = saved
        return out

    def advance(self, n):
        for _ in range(n):
            self._next_word()

    def state_words(self):
        """The 34 most recent words, oldest first (orbx_rand_state.r with i = 34)."""
        return list(self._r[-34:])

    def set_state_words(self, words):
        self._r = [int(w) & 0xFFFFFFFF for w in words][-34:]
