"""CPU restatement of the reference's random formation-group generator
(SURVEY.md §8f row 4).

TEST INFRASTRUCTURE ONLY: the checker of acl_generate_formation_groups; the
product never imports it.

Reference: aclswarm_sim/nodes/generate_random_formation.py
  sample_point (:20-24)              x, y, z = uniform(-l/2, l/2),
                                     uniform(-w/2, w/2), uniform(0, h)
  generate_formation (:26-56)        rejection: a point closer than min_dist
                                     (xy) to an accepted one is discarded
  generate_formation_group (:59-80)  adjmat = ones - eye; unless fc:
                                     m = randint(1, n - 4 + 1),
                                     rowIdx = choice(n, m), colIdx = choice(n, m)
                                     (with replacement), adj[r][c] = adj[c][r] = 0;
                                     then formations 'A' and 'B'
seeded with np.random.seed(s) (trial.sh:60).

Third-party algorithm: numpy's legacy RandomState (numpy 2.2 here; the
reference pins none). Restated from its published semantics:
  * seed(int s): MT19937 init_genrand(s & 0xffffffff) (mt19937_seed);
  * next_uint32: MT19937 genrand_int32 (twist every 624 outputs, tempering);
  * next_double: (a >> 5) * 67108864 + (b >> 6), / 2**53 (two outputs);
  * uniform(low, high): low + (high - low) * next_double;
  * randint(low, high) and choice(n, size) with replacement: masked
    rejection on 32-bit outputs, mask = 2**k - 1 >= rng = high - 1 - low,
    redraw while (u & mask) > rng; rng == 0 draws nothing.
Pinned by tests/test_formation_gen.py: against numpy's own RandomState on the
same seeds, and against tests/golden/simform*.npz (made by importing the
reference generator, tests/golden/make_fixtures.py) bit for bit. The
reference's 5 s wall-clock timeout (:35-53) has no counterpart: a group that
needs more than `max_candidates` samples per formation is reported instead.
"""
import math


class MT19937:
    N, M = 624, 397

    def __init__(self, seed):
        mt = [0] * self.N
        s = seed & 0xFFFFFFFF
        for i in range(self.N):
            mt[i] = s
            s = (1812433253 * (s ^ (s >> 30)) + i + 1) & 0xFFFFFFFF
        self.mt = mt
        self.pos = self.N
        self.drawn = 0

    def _twist(self):
        mt, N, M = self.mt, self.N, self.M
        for i in range(N):
            y = (mt[i] & 0x80000000) | (mt[(i + 1) % N] & 0x7FFFFFFF)
            mt[i] = mt[(i + M) % N] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
        self.pos = 0

    def next_uint32(self):
        if self.pos >= self.N:
            self._twist()
        y = self.mt[self.pos]
        self.pos += 1
        self.drawn += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y

    def next_double(self):
        a = self.next_uint32() >> 5
        b = self.next_uint32() >> 6
        return (a * 67108864.0 + b) / 9007199254740992.0

    def uniform(self, low, high):
        return low + (high - low) * self.next_double()

    def bounded(self, rng):
        """masked rejection in [0, rng] (numpy buffered_bounded_masked_uint32)."""
        if rng == 0:
            return 0
        mask = rng
        for sh in (1, 2, 4, 8, 16):
            mask |= mask >> sh
        while True:
            v = self.next_uint32() & mask
            if v <= rng:
                return v


def generate_formation(rs, n, l, w, h, min_dist, max_candidates=10 ** 7):
    r = min_dist / 2.0
    pts = []
    tries = 0
    while len(pts) < n:
        x = rs.uniform(-l / 2.0, l / 2.0)
        y = rs.uniform(-w / 2.0, w / 2.0)
        z = rs.uniform(0.0, h)
        tries += 1
        ok = True
        for p in pts:
            dx, dy = x - p[0], y - p[1]
            if math.sqrt(dx * dx + dy * dy) < 2 * r:
                ok = False
                break
        if ok:
            pts.append((x, y, z))
        if tries > max_candidates:
            return None
    return pts


def generate_formation_group(seed, n, fc, l, w, h, min_dist):
    """-> (adjmat [n][n] list of 0/1, [points A, points B], outputs drawn)."""
    rs = MT19937(seed)
    adj = [[0 if i == j else 1 for j in range(n)] for i in range(n)]
    if not fc:
        m = 1 + rs.bounded(n - 4 + 1 - 1 - 1)      # randint(1, n - 4 + 1)
        rows = [rs.bounded(n - 1) for _ in range(m)]  # choice(n, size=(m,))
        cols = [rs.bounded(n - 1) for _ in range(m)]
        for i in range(m):
            adj[rows[i]][cols[i]] = 0
            adj[cols[i]][rows[i]] = 0
    forms = [generate_formation(rs, n, l, w, h, min_dist) for _ in range(2)]
    return adj, forms, rs.drawn
