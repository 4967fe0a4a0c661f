// formation_gen.hip -- the reference's random formation-group generator on
// the device, stream-exact.
//
// aclswarm_sim/nodes/generate_random_formation.py:20-96 seeded with
// np.random.seed(s) (trial.sh:60): numpy's legacy RandomState = MT19937
// (init_genrand seeding), uniform doubles from two 32-bit outputs, masked
// rejection for randint / choice. One wavefront per formation group:
//
//   * the generator state lives in LDS as two consecutive 624-word blocks of
//     the MT19937 sequence (current, next), so any window of up to 624
//     outputs past the read position is addressable; a twist computes the
//     next block from the current one in three lane-parallel phases
//     (i < 227 reads the old block only, 227 <= i < 454 and i >= 454 read
//     the new words 227 positions back);
//   * bounded draws (randint / choice): 64 lanes test 64 consecutive outputs,
//     a ballot finds the first accepted one;
//   * rejection sampling of points: 64 lanes take 64 consecutive candidates
//     (6 outputs each), test them against the accepted points in parallel,
//     then resolve the batch in candidate order with ballots (a candidate is
//     accepted iff it clears the points accepted before it), and the read
//     position advances past the candidate that completed the formation.
//
// All arithmetic is the reference's operation for operation (-ffp-contract=off),
// so points are bit-identical to the CPU generator's; tests/test_gpu_formation_gen.py
// checks them against tests/golden/simform*.npz (the reference's own output).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/aclswarm_amd.h"

extern "C" acl_status_t acl__set_error(const char* msg);

namespace acl_amd {

constexpr int kMtN = 624, kMtM = 397;

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= y >> 11;
  y ^= (y << 7) & 0x9D2C5680u;
  y ^= (y << 15) & 0xEFC60000u;
  y ^= y >> 18;
  return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b) {
  const uint32_t y = (a & 0x80000000u) | (b & 0x7FFFFFFFu);
  return (y >> 1) ^ ((y & 1u) ? 0x9908B0DFu : 0u);
}

// out = the MT19937 block that follows `in` (genrand_int32's in-place twist)
__device__ void mt_twist(const uint32_t* in, uint32_t* out, int lane) {
  for (int i = lane; i < 227; i += 64) out[i] = in[i + kMtM] ^ mt_mix(in[i], in[i + 1]);
  __syncthreads();
  for (int i = 227 + lane; i < 454; i += 64) out[i] = out[i - 227] ^ mt_mix(in[i], in[i + 1]);
  __syncthreads();
  for (int i = 454 + lane; i < kMtN; i += 64)
    out[i] = out[i - 227] ^ mt_mix(in[i], i + 1 < kMtN ? in[i + 1] : out[0]);
  __syncthreads();
}

struct MtStream {
  uint32_t* buf[2];  // buf[cur]: current block, buf[cur ^ 1]: the next one
  int cur;
  int pos;           // read position in the current block
  long long drawn;

  __device__ uint32_t raw(int k) const {  // k-th output past pos, k < 624
    const int a = pos + k;
    return a < kMtN ? buf[cur][a] : buf[cur ^ 1][a - kMtN];
  }
  __device__ uint32_t out(int k) const { return mt_temper(raw(k)); }
  __device__ void advance(int cnt, int lane) {
    pos += cnt;
    drawn += cnt;
    while (pos >= kMtN) {
      pos -= kMtN;
      cur ^= 1;
      mt_twist(buf[cur], buf[cur ^ 1], lane);
    }
  }
};

// numpy next_double: ((a >> 5) * 67108864 + (b >> 6)) / 2^53
__device__ __forceinline__ double mt_double(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}

// buffered_bounded_masked_uint32: the first output with (u & mask) <= rng
__device__ uint32_t mt_bounded(MtStream& S, uint32_t rng, int lane) {
  if (rng == 0u) return 0u;
  uint32_t mask = rng;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
  for (;;) {
    const uint32_t u = S.out(lane) & mask;
    const unsigned long long ok = __ballot(u <= rng);
    if (ok) {
      const int first = __ffsll((long long)ok) - 1;
      const uint32_t v = (uint32_t)__shfl((int)u, first, 64);
      S.advance(first + 1, lane);
      return v;
    }
    S.advance(64, lane);
  }
}

struct GenParams {
  int F, n, fc;
  const uint32_t* seeds;
  double l, w, h, min_dist;
  long long max_candidates;
  double* points;     // [F][2][n][3]
  uint8_t* adj;       // [F][n][n]
  int32_t* status;    // [F]
  long long* drawn;   // [F] (optional)
};

__global__ void __launch_bounds__(64) formation_gen_kernel(const GenParams P) {
  __shared__ uint32_t blk[2][kMtN];
  __shared__ int s_rc[512];
  extern __shared__ double acc_xy[];  // [n][2] accepted points of the formation
  const int g = blockIdx.x, lane = threadIdx.x, n = P.n;
  // np.random.seed(s): init_genrand into blk[1]
  if (lane == 0) {
    uint32_t s = P.seeds[g];
    for (int i = 0; i < kMtN; ++i) {
      blk[1][i] = s;
      s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
    }
  }
  __syncthreads();
  // the seeded state has pos = 624: the first draw twists. blk[0] = outputs
  // 0..623 (untempered), blk[1] = outputs 624..1247
  mt_twist(blk[1], blk[0], lane);
  mt_twist(blk[0], blk[1], lane);
  MtStream S;
  S.buf[0] = blk[0];
  S.buf[1] = blk[1];
  S.cur = 0;
  S.pos = 0;
  S.drawn = 0;

  // adjacency: ones - eye, minus m random pairs (generate_formation_group :61-72)
  uint8_t* A = P.adj + (size_t)g * n * n;
  for (int k = lane; k < n * n; k += 64) A[k] = (k / n == k % n) ? 0 : 1;
  __syncthreads();
  if (!P.fc) {
    const int m = 1 + (int)mt_bounded(S, (uint32_t)(n - 5), lane);  // randint(1, n - 4 + 1)
    for (int i = 0; i < m; ++i) {
      const int r = (int)mt_bounded(S, (uint32_t)(n - 1), lane);    // choice(n, size=(m,))
      if (lane == 0) s_rc[i] = r;
    }
    for (int i = 0; i < m; ++i) {
      const int c = (int)mt_bounded(S, (uint32_t)(n - 1), lane);
      if (lane == 0) {
        const int r = s_rc[i];
        A[(size_t)r * n + c] = 0;
        A[(size_t)c * n + r] = 0;
      }
    }
  }
  // formations 'A' and 'B' (generate_formation :26-56)
  const double lo_x = -P.l / 2.0, hi_x = P.l / 2.0;
  const double lo_y = -P.w / 2.0, hi_y = P.w / 2.0;
  const double lo_z = 0.0, hi_z = P.h;
  const double two_r = 2 * (P.min_dist / 2.0);
  int status = 0;
  for (int fm = 0; fm < 2 && !status; ++fm) {
    double* out = P.points + ((size_t)g * 2 + fm) * n * 3;
    int na = 0;
    long long tried = 0;
    while (na < n) {
      // candidate `lane`: outputs 6 lane .. 6 lane + 5 past the read position
      const double x = lo_x + (hi_x - lo_x) * mt_double(S.out(6 * lane), S.out(6 * lane + 1));
      const double y = lo_y + (hi_y - lo_y) * mt_double(S.out(6 * lane + 2), S.out(6 * lane + 3));
      const double z = lo_z + (hi_z - lo_z) * mt_double(S.out(6 * lane + 4), S.out(6 * lane + 5));
      bool pre = true;
      for (int k = 0; k < na; ++k) {
        const double dx = x - acc_xy[2 * k], dy = y - acc_xy[2 * k + 1];
        if (sqrt(dx * dx + dy * dy) < two_r) pre = false;
      }
      // candidates in order: accepted iff clear of the points accepted before
      bool acc = false;
      int last = 63, need = n - na;
      const unsigned long long prem = __ballot(pre);
      for (int c = 0; c < 64; ++c) {
        if (!((prem >> c) & 1ull)) continue;
        const double xc = __shfl(x, c, 64), yc = __shfl(y, c, 64);
        const double dx = x - xc, dy = y - yc;
        const bool clash = acc && lane < c && sqrt(dx * dx + dy * dy) < two_r;
        if (__ballot(clash) == 0ull) {
          if (lane == c) acc = true;
          if (--need == 0) {
            last = c;
            break;
          }
        }
      }
      // append the accepted candidates in candidate order
      const unsigned long long am = __ballot(acc);
      if (acc) {
        const int slot = na + __popcll(am & ((1ull << lane) - 1ull));
        acc_xy[2 * slot] = x;
        acc_xy[2 * slot + 1] = y;
        out[3 * slot] = x;
        out[3 * slot + 1] = y;
        out[3 * slot + 2] = z;
      }
      na += __popcll(am);
      __syncthreads();
      S.advance(6 * (last + 1), lane);
      tried += last + 1;
      if (na < n && tried > P.max_candidates) {
        status |= 1 << fm;  // the reference's 5 s timeout returns {} here
        break;
      }
    }
  }
  if (lane == 0) {
    P.status[g] = status;
    if (P.drawn) P.drawn[g] = S.drawn;
  }
}

}  // namespace acl_amd

extern "C" acl_status_t acl_generate_formation_groups(int32_t F, int32_t n, const uint32_t* seeds,
                                                      int32_t fc, double l, double w, double h,
                                                      double min_dist, int64_t max_candidates,
                                                      double* points, uint8_t* adj,
                                                      int32_t* status, int64_t* drawn,
                                                      void* stream) {
  using namespace acl_amd;
  if (F < 0 || n < 1 || n > 512)
    return acl__set_error("acl_generate_formation_groups: F < 0 or n out of range [1, 512]");
  if (!fc && n < 5)
    return acl__set_error("acl_generate_formation_groups: a noncomplete group needs n >= 5 "
                          "(randint(1, n - 3), generate_random_formation.py:64)");
  if (F == 0) return ACL_OK;
  if (!seeds || !points || !adj || !status)
    return acl__set_error("acl_generate_formation_groups: required pointer is NULL");
  GenParams P;
  P.F = F; P.n = n; P.fc = fc; P.seeds = seeds; P.l = l; P.w = w; P.h = h;
  P.min_dist = min_dist; P.max_candidates = max_candidates > 0 ? max_candidates : 10000000;
  P.points = points; P.adj = adj; P.status = status; P.drawn = (long long*)drawn;
  hipLaunchKernelGGL(formation_gen_kernel, dim3(F), dim3(64), (size_t)n * 2 * sizeof(double),
                     (hipStream_t)stream, P);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? ACL_OK : acl__set_error(hipGetErrorString(e));
}
