// control.hip -- batched DistCntrl::compute + Safety for gfx950.
//
// Runs after the auction kernel (solve.hip) on the same swarms, on a second
// stream so that one chunk's gain stream overlaps the next chunk's auction.
// Two kernels:
//
//   gain_kernel    DistCntrl::compute (aclswarm/src/distcntrl.cpp:46-102):
//                  the HBM stream (72 B of gain block per directed edge).
//                  One wave per vehicle v, lanes = formation neighbours j of
//                  v's adopted point i (two chunks of 64), the 3x3 block A_ij
//                  read from the 9 coalesced planes, pdistmat's Gram-formula
//                  distances (utils.h:137-147), atan scale terms gated on
//                  |e| > thr, per-neighbour damping; a wave sum gives u (tree
//                  order: parity within 1e-5 relative). Lean on registers and
//                  LDS (~7 KB per swarm) so 8 swarms are resident per CU and
//                  enough gain bytes are in flight.
//   safety_kernel  Safety::cmdinCb saturation (safety.cpp:185-196) and
//                  Safety::collisionAvoidance (safety.cpp:412-541): lanes find
//                  the vehicles inside d_avoid_thresh, lane 0 sorts the sector
//                  edges, unions them and picks the closest safe edge exactly
//                  as the reference.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/aclswarm_amd.h"
#include "common.h"
#include "control_params.h"

namespace acl_amd {

constexpr int kCtlBlock = 256;
constexpr int kCtlWaves = kCtlBlock / 64;

__host__ __device__ inline int cal16(int x) { return (x + 15) & ~15; }

struct GainLayout {
  int q, p, adjF, rowptr, Pt, myi, out, total;
};

__host__ __device__ inline GainLayout make_gain_layout(int n) {
  GainLayout L;
  int o = 0;
  L.q = o;      o = cal16(o + n * 3 * 8);
  L.p = o;      o = cal16(o + n * 3 * 8);
  L.adjF = o;   o = cal16(o + n * 2 * 8);
  L.rowptr = o; o = cal16(o + (n + 1) * 4);
  L.Pt = o;     o = cal16(o + n);
  L.myi = o;    o = cal16(o + n);
  L.out = o;    o = cal16(o + n * 3 * 8);
  L.total = o;
  return L;
}

__global__ void __launch_bounds__(kCtlBlock, 4) gain_kernel(const CtlParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = P.n;
  const GainLayout L = make_gain_layout(n);
  const int b = P.b0 + blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  if (P.status[b].flags & ACL_SWARM_BAD_INPUT) return;  // auction kernel zeroed outputs

  double* q = reinterpret_cast<double*>(smem + L.q);
  double* p = reinterpret_cast<double*>(smem + L.p);
  unsigned long long* adjF = reinterpret_cast<unsigned long long*>(smem + L.adjF);
  int* rowptr = reinterpret_cast<int*>(smem + L.rowptr);
  unsigned char* Pt = smem + L.Pt;
  unsigned char* myi = smem + L.myi;
  double* uo = reinterpret_cast<double*>(smem + L.out);

  const int f = P.fidx[b];
  const int gw = (n + 63) >> 6;
  const unsigned long long lastmask = (n & 63) ? ((1ull << (n & 63)) - 1ull) : ~0ull;
  const bool uniform = P.ws[(size_t)P.B * n + b] == 0;
  const unsigned char* rows = P.ws + (size_t)P.B * (n + 1) + (size_t)b * n * n;
  {
    const double* gq = P.q + (size_t)b * n * 3;
    const double* gp = P.p + (size_t)f * n * 3;
    for (int k = tid; k < 3 * n; k += kCtlBlock) {
      q[k] = gq[k];
      p[k] = gp[k];
    }
    const uint64_t* ga = P.adj + (size_t)f * n * gw;
    for (int k = tid; k < n * 2; k += kCtlBlock) {
      const int i = k >> 1, w = k & 1;
      unsigned long long x = 0;
      if (w < gw) {
        x = ga[(size_t)i * gw + w];
        if (w == gw - 1) x &= lastmask;
      }
      adjF[k] = x;
    }
    for (int v = tid; v < n; v += kCtlBlock) {
      myi[v] = (unsigned char)P.P_out[(size_t)b * n + v];
      if (uniform) Pt[v] = P.ws[(size_t)b * n + v];
    }
  }
  __syncthreads();
  // formation CSR row starts (edges enumerated row-major, diagonal included)
  if (wave == 0) {
    int base = 0;
    for (int c = 0; c < 2; ++c) {
      const int i = lane + 64 * c;
      const int cnt = (i < n) ? __popcll(adjF[2 * i]) + __popcll(adjF[2 * i + 1]) : 0;
      int x = cnt;  // inclusive wave scan
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (i < n) rowptr[i] = base + x - cnt;
      base += __shfl(x, 63, 64);
    }
    if (lane == 0) rowptr[n] = base;
  }
  __syncthreads();

  const int E = rowptr[n];
  const double* G = P.gains + 9 * P.gain_off[f];
  const acl_cntrl_gains_t g = P.g;
  for (int v = wave; v < n; v += kCtlWaves) {
    const int i = myi[v];
    const double* gv = P.vel + ((size_t)b * n + v) * 3;
    const double vel0 = gv[0], vel1 = gv[1], vel2 = gv[2];
    const double qv0 = q[3 * v], qv1 = q[3 * v + 1], qv2 = q[3 * v + 2];
    const double pix = p[3 * i], piy = p[3 * i + 1], piz = p[3 * i + 2];
    const double Ni = pix * pix + piy * piy, Nzi = piz * piz;
    double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
    int ebase = rowptr[i];
#pragma unroll 1
    for (int c = 0; c < 2; ++c) {
      const unsigned long long rowbits = adjF[2 * i + c];
      const bool has = (rowbits >> lane) & 1ull;
      const int e = ebase + __popcll(rowbits & ((1ull << lane) - 1ull));
      ebase += __popcll(rowbits);
      if (has) {
        double A[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) A[k] = __builtin_nontemporal_load(G + (size_t)k * E + e);
        const int j = lane + 64 * c;
        const int uu = uniform ? Pt[j] : rows[(size_t)v * n + j];
        const double q0 = q[3 * uu] - qv0, q1 = q[3 * uu + 1] - qv1, q2 = q[3 * uu + 2] - qv2;
        const double pjx = p[3 * j], pjy = p[3 * j + 1], pjz = p[3 * j + 2];
        const double Nj = pjx * pjx + pjy * pjy, Nzj = pjz * pjz;
        const double dxy = sqrt((Ni + Nj) - 2.0 * (pix * pjx + piy * pjy));
        const double dz = sqrt((Nzi + Nzj) - 2.0 * (piz * pjz));
        const double e_xy = sqrt(q0 * q0 + q1 * q1) - dxy;
        const double e_z = sqrt(q2 * q2) - dz;
        double Fxy = 0.0, Fz = 0.0;
        if (fabs(e_xy) > g.e_xy_thr) Fxy = g.K1_xy * acl_atan(g.K2_xy * e_xy);
        if (fabs(e_z) > g.e_z_thr) Fz = g.K1_z * acl_atan(g.K2_z * e_z);
        const double up0 = ((A[0] * q0 + A[1] * q1) + A[2] * q2) + Fxy * q0;
        const double up1 = ((A[3] * q0 + A[4] * q1) + A[5] * q2) + Fxy * q1;
        const double up2 = ((A[6] * q0 + A[7] * q1) + A[8] * q2) + Fz * q2;
        acc0 += g.kp * up0 + g.kd * (-vel0);
        acc1 += g.kp * up1 + g.kd * (-vel1);
        acc2 += g.kp * up2 + g.kd * (-vel2);
      }
    }
    const double cmd0 = wave_sum(acc0), cmd1 = wave_sum(acc1), cmd2 = wave_sum(acc2);
    if (lane == 0) {
      uo[3 * v] = cmd0; uo[3 * v + 1] = cmd1; uo[3 * v + 2] = cmd2;
    }
  }
  __syncthreads();
  for (int k = tid; k < 3 * n; k += kCtlBlock) P.u[(size_t)b * n * 3 + k] = uo[k];
}

struct SafeLayout {
  int q, u, caA, caS, misc, total;
};

__host__ __device__ inline SafeLayout make_safe_layout(int n) {
  SafeLayout L;
  int o = 0;
  L.q = o;    o = cal16(o + n * 3 * 8);
  L.u = o;    o = cal16(o + n * 3 * 8);
  L.caA = o;  o = cal16(o + kCtlWaves * 4 * n * 8);
  L.caS = o;  o = cal16(o + kCtlWaves * 4 * n);
  L.misc = o; o = cal16(o + 16);
  L.total = o;
  return L;
}

__global__ void __launch_bounds__(kCtlBlock) safety_kernel(const CtlParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int n = P.n;
  const SafeLayout L = make_safe_layout(n);
  const int b = P.b0 + blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  if (P.status[b].flags & ACL_SWARM_BAD_INPUT) return;

  double* q = reinterpret_cast<double*>(smem + L.q);
  double* uo = reinterpret_cast<double*>(smem + L.u);
  int* misc = reinterpret_cast<int*>(smem + L.misc);
  {
    const double* gq = P.q + (size_t)b * n * 3;
    const double* gu = P.u + (size_t)b * n * 3;
    for (int k = tid; k < 3 * n; k += kCtlBlock) {
      q[k] = gq[k];
      uo[k] = gu[k];
    }
    if (tid == 0) misc[0] = 0;
  }
  __syncthreads();
  const acl_safety_params_t sp = P.s;
  double* caA = reinterpret_cast<double*>(smem + L.caA) + wave * (4 * n);
  signed char* caS = reinterpret_cast<signed char*>(smem + L.caS) + wave * (4 * n);
  int nca = 0;
  for (int v = wave; v < n; v += kCtlWaves) {
    double cmd0 = uo[3 * v], cmd1 = uo[3 * v + 1], cmd2 = uo[3 * v + 2];
    const double qv0 = q[3 * v], qv1 = q[3 * v + 1];
    // Safety::cmdinCb saturation (safety.cpp:185-196)
    {
      const double velxy = sqrt(cmd0 * cmd0 + cmd1 * cmd1);
      if (velxy > sp.max_vel_xy) {
        cmd0 = cmd0 / velxy * sp.max_vel_xy;
        cmd1 = cmd1 / velxy * sp.max_vel_xy;
      }
      const double velz = fabs(cmd2);
      if (velz > sp.max_vel_z) cmd2 = cmd2 / velz * sp.max_vel_z;
    }
    // Safety::collisionAvoidance (safety.cpp:412-541)
    bool modified = false;
    {
      bool cand[2];
      double dxv[2], dyv[2], dv[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int j = lane + 64 * c;
        cand[c] = false;
        dxv[c] = dyv[c] = dv[c] = 0.0;
        if (j < n && j != v) {
          dxv[c] = q[3 * j] - qv0;
          dyv[c] = q[3 * j + 1] - qv1;
          dv[c] = sqrt(dxv[c] * dxv[c] + dyv[c] * dyv[c]);
          cand[c] = !(dv[c] > sp.d_avoid_thresh);
        }
      }
      const unsigned long long m0 = __ballot(cand[0]), m1 = __ballot(cand[1]);
      if (m0 | m1) {
        bool wrapped = false;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          if (cand[c]) {
            const int slot = 4 * (__popcll((c ? m1 : m0) & ((1ull << lane) - 1ull)) +
                                  (c ? __popcll(m0) : 0));
            const double theta = atan2(dyv[c], dxv[c]);
            const double x = sp.r_keep_out / dv[c];
            const double alpha = fabs(asin(x < 1.0 ? x : 1.0));
            const double beg = wrap_to_pi(theta - alpha);
            const double end = wrap_to_pi(theta + alpha);
            caA[slot] = beg;     caS[slot] = +1;
            caA[slot + 1] = end; caS[slot + 1] = -1;
            if (beg > end) {
              wrapped = true;
              caA[slot + 2] = -kPi; caS[slot + 2] = +1;
              caA[slot + 3] = kPi;  caS[slot + 3] = -1;
            } else {
              caS[slot + 2] = 0;
              caS[slot + 3] = 0;
            }
          }
        }
        const bool didWrap = __any(wrapped);
        const int nslot = 4 * (__popcll(m0) + __popcll(m1));
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
        if (lane == 0) {
          // compact + insertion sort by (angle, sign) = std::sort on pairs
          int ne = 0;
          for (int k = 0; k < nslot; ++k) {
            const signed char sg = caS[k];
            if (sg == 0) continue;
            const double a = caA[k];
            int pos = ne;
            while (pos > 0 && (a < caA[pos - 1] || (!(caA[pos - 1] < a) && sg < caS[pos - 1]))) {
              caA[pos] = caA[pos - 1];
              caS[pos] = caS[pos - 1];
              --pos;
            }
            caA[pos] = a;
            caS[pos] = sg;
            ++ne;
          }
          // parenthesis-count union into zones, stored in place (nz <= ne/2)
          int nz = 0, count = 0;
          double start = 0.0;
          for (int k = 0; k < ne; ++k) {
            const double a = caA[k];
            if (count == 0) start = a;
            count += caS[k];
            if (count == 0) {
              caA[2 * nz] = start;
              caA[2 * nz + 1] = a;
              ++nz;
            }
          }
          const double psi = atan2(cmd1, cmd0);
          bool safe = true;
          for (int k = 0; k < nz; ++k)
            if (psi > caA[2 * k] && psi < caA[2 * k + 1]) { safe = false; break; }
          if (!safe) {
            modified = true;
            // flatten zone edges (drop +-pi ones when wrapped), sort
            int m = 0;
            for (int k = 0; k < 2 * nz; ++k) {
              const double a = caA[k];
              if (!didWrap || fabs(a) != kPi) caA[m++] = a;
            }
            if (m == 0) {
              cmd0 = cmd1 = 0.0;
              cmd2 = 0.0;
            } else {
              for (int k = 1; k < m; ++k) {
                const double a = caA[k];
                int pos = k;
                while (pos > 0 && a < caA[pos - 1]) { caA[pos] = caA[pos - 1]; --pos; }
                caA[pos] = a;
              }
              int it = 0;  // std::lower_bound
              while (it < m && caA[it] < psi) ++it;
              int idx;
              if (it == 0) idx = 0;
              else if (it == m || fabs(caA[it - 1] - psi) < fabs(caA[it] - psi)) idx = it - 1;
              else idx = it;
              const double edge = caA[idx];
              if (fabs(wrap_to_pi(edge - psi)) <= kPi / 2) {
                const double umag = sqrt(cmd0 * cmd0 + cmd1 * cmd1);
                cmd0 = umag * cos(edge);
                cmd1 = umag * sin(edge);
              } else {
                cmd0 = cmd1 = 0.0;
                cmd2 = 0.0;
              }
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" ::: "memory");
      }
    }
    if (lane == 0) {
      uo[3 * v] = cmd0; uo[3 * v + 1] = cmd1; uo[3 * v + 2] = cmd2;
      if (P.ca_flag) P.ca_flag[(size_t)b * n + v] = modified;
      nca += modified;
    }
  }
  if (lane == 0 && nca) atomicAdd(&misc[0], nca);
  __syncthreads();
  if (P.u_safe)
    for (int k = tid; k < 3 * n; k += kCtlBlock) P.u_safe[(size_t)b * n * 3 + k] = uo[k];
  if (tid == 0 && misc[0]) {
    P.status[b].n_ca = (uint16_t)misc[0];
    P.status[b].flags |= ACL_SWARM_CA_ACTIVE;
  }
}

hipError_t launch_control(const CtlParams& P, int nb, int which, hipStream_t stream) {
  if (which == 0) {
    const GainLayout L = make_gain_layout(P.n);
    hipLaunchKernelGGL(gain_kernel, dim3(nb), dim3(kCtlBlock), L.total, stream, P);
  } else {
    const SafeLayout L = make_safe_layout(P.n);
    hipLaunchKernelGGL(safety_kernel, dim3(nb), dim3(kCtlBlock), L.total, stream, P);
  }
  return hipGetLastError();
}

}  // namespace acl_amd
