// common.h -- device helpers shared by the auction and control kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace acl_amd {

constexpr double kPi = 3.14159265358979323846;

// Wave64 reductions on DPP (VALU lane shuffles, no LDS round trip):
// quad_perm [1,0,3,2], [2,3,0,1], row_ror 4, 8 give every lane its row's
// result; row_bcast15 / row_bcast31 fold rows 0-3 into lane 63.
// Callers must have all 64 lanes active.
// DPP lane move with the reduction identity 0 in lanes the pattern leaves
// out (bound_ctrl): `op(x, dppz<..>(x))` folds into one `v_op_dpp`.
template <int CTRL, int RMASK>
__device__ __forceinline__ unsigned dppz(unsigned x) {
  return (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, RMASK, 0xF, true);
}

// Result of a 6-step wave reduction sits in lane 63.
#define ACL_WAVE_REDUCE(x, OP)          \
  x = OP(x, dppz<0xB1, 0xF>(x));        \
  x = OP(x, dppz<0x4E, 0xF>(x));        \
  x = OP(x, dppz<0x124, 0xF>(x));       \
  x = OP(x, dppz<0x128, 0xF>(x));       \
  x = OP(x, dppz<0x142, 0xA>(x));       \
  x = OP(x, dppz<0x143, 0xC>(x))

__device__ __forceinline__ unsigned op_umax(unsigned a, unsigned b) { return a > b ? a : b; }
__device__ __forceinline__ unsigned op_or(unsigned a, unsigned b) { return a | b; }

__device__ __forceinline__ unsigned wave_max_u32(unsigned x) {
  ACL_WAVE_REDUCE(x, op_umax);
  return (unsigned)__builtin_amdgcn_readlane((int)x, 63);
}

__device__ __forceinline__ unsigned wave_or_u32(unsigned x) {
  ACL_WAVE_REDUCE(x, op_or);
  return (unsigned)__builtin_amdgcn_readlane((int)x, 63);
}

// non-negative floats order like their bit patterns
__device__ __forceinline__ float wave_max_f32_nonneg(float fx) {
  return __uint_as_float(wave_max_u32(__float_as_uint(fx)));
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long x) {
  const unsigned hi = (unsigned)(x >> 32), lo = (unsigned)x;
  const unsigned mh = wave_max_u32(hi);
  const unsigned ml = wave_max_u32(hi == mh ? lo : 0u);
  return ((unsigned long long)mh << 32) | ml;
}

// DPP move of a double; lanes outside RMASK read 0 (the sum's identity).
template <int CTRL, int RMASK>
__device__ __forceinline__ double dpp_f64_z(double x) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)u, CTRL, RMASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), CTRL, RMASK, 0xF, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

// Sum over the wave, result in every lane (tree order: the control law's
// parity is tolerance-based, 1e-5 relative).
__device__ __forceinline__ double wave_sum(double x) {
  x += dpp_f64_z<0xB1, 0xF>(x);
  x += dpp_f64_z<0x4E, 0xF>(x);
  x += dpp_f64_z<0x124, 0xF>(x);
  x += dpp_f64_z<0x128, 0xF>(x);
  x += dpp_f64_z<0x142, 0xA>(x);
  x += dpp_f64_z<0x143, 0xC>(x);
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)u, 63);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(u >> 32), 63);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// atan in fp64, branch-free (selects): the classic fdlibm reduction to
// |t| < 7/16 around atan(0.5), atan(1), atan(1.5), atan(inf) and its odd
// degree-23 polynomial; max error 1 ulp (checked against libm on 3e5 points).
// Leaner in registers than the library call, which matters in the gain
// kernel's occupancy.
__device__ __forceinline__ double acl_atan(double x) {
  const double ax = fabs(x);
  const bool r0 = ax >= 0.4375, r1 = ax >= 0.6875, r2 = ax >= 1.1875, r3 = ax >= 2.4375;
  double num = ax, den = 1.0, hi = 0.0, lo = 0.0;
  if (r0) { num = 2.0 * ax - 1.0; den = 2.0 + ax; hi = 4.63647609000806093515e-01; lo = 2.26987774529616870924e-17; }
  if (r1) { num = ax - 1.0; den = ax + 1.0; hi = 7.85398163397448278999e-01; lo = 3.06161699786838301793e-17; }
  if (r2) { num = ax - 1.5; den = 1.0 + 1.5 * ax; hi = 9.82793723247329054082e-01; lo = 1.39033110312309984516e-17; }
  if (r3) { num = -1.0; den = ax; hi = 1.57079632679489655800e+00; lo = 6.12323399573676603587e-17; }
  const double t = num / den;
  const double z = t * t, w = z * z;
  const double s1 = z * (3.33333333333329318027e-01 + w * (1.42857142725034663711e-01 +
                    w * (9.09088713343650656196e-02 + w * (6.66107313738753120669e-02 +
                    w * (4.97687799461593236017e-02 + w * 1.62858201153657823623e-02)))));
  const double s2 = w * (-1.99999999998764832476e-01 + w * (-1.11111104054623557880e-01 +
                    w * (-7.69187620504482999495e-02 + w * (-5.83357013379057348645e-02 +
                    w * -3.65315727442169155270e-02))));
  const double r = r0 ? hi - ((t * (s1 + s2) - lo) - t) : t - t * (s1 + s2);
  return copysign(r, x);
}

// A wave-uniform double moved to SGPRs (two v_readfirstlane).
__device__ __forceinline__ double uni(double x) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(x);
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)u);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ unsigned long long uni_u64(unsigned long long u) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)u);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(u >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

// Fast fp64 kernels for the control law, whose parity is tolerance-based
// (1e-5 relative): a square root from v_rsq_f64 refined by one Goldschmidt
// step and a correction (about 1 ulp for normal inputs; 0, +inf and
// negative inputs as IEEE sqrt), and a quotient from v_rcp_f64 refined by
// two Newton steps (about 1 ulp; den finite and nonzero).
__device__ __forceinline__ double sqrt_nr(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = __builtin_fma(-g, h, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  const double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  return (x == 0.0 || __builtin_isinf(x)) ? x : g;
}

__device__ __forceinline__ double div_nr(double num, double den) {
  double r = __builtin_amdgcn_rcp(den);
  r = __builtin_fma(__builtin_fma(-den, r, 1.0), r, r);
  r = __builtin_fma(__builtin_fma(-den, r, 1.0), r, r);
  const double q = num * r;
  return __builtin_fma(__builtin_fma(-den, q, num), r, q);
}

// acl_atan with the fast quotient and fused multiply-adds (control law only).
__device__ __forceinline__ double acl_atan_fast(double x) {
  const double ax = fabs(x);
  const bool r0 = ax >= 0.4375, r1 = ax >= 0.6875, r2 = ax >= 1.1875, r3 = ax >= 2.4375;
  double num = ax, den = 1.0, hi = 0.0, lo = 0.0;
  if (r0) { num = 2.0 * ax - 1.0; den = 2.0 + ax; hi = 4.63647609000806093515e-01; lo = 2.26987774529616870924e-17; }
  if (r1) { num = ax - 1.0; den = ax + 1.0; hi = 7.85398163397448278999e-01; lo = 3.06161699786838301793e-17; }
  if (r2) { num = ax - 1.5; den = 1.0 + 1.5 * ax; hi = 9.82793723247329054082e-01; lo = 1.39033110312309984516e-17; }
  if (r3) { num = -1.0; den = ax; hi = 1.57079632679489655800e+00; lo = 6.12323399573676603587e-17; }
  const double t = r0 ? div_nr(num, den) : ax;
  const double z = t * t, w = z * z;
  const double s1 = z * __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, __builtin_fma(w,
                    __builtin_fma(w, 1.62858201153657823623e-02, 4.97687799461593236017e-02),
                    6.66107313738753120669e-02), 9.09088713343650656196e-02),
                    1.42857142725034663711e-01), 3.33333333333329318027e-01);
  const double s2 = w * __builtin_fma(w, __builtin_fma(w, __builtin_fma(w,
                    __builtin_fma(w, -3.65315727442169155270e-02, -5.83357013379057348645e-02),
                    -7.69187620504482999495e-02), -1.11111104054623557880e-01),
                    -1.99999999998764832476e-01);
  const double r = r0 ? hi - (__builtin_fma(t, s1 + s2, -lo) - t) : __builtin_fma(-t, s1 + s2, t);
  return (ax == __builtin_inf()) ? copysign(1.57079632679489655800e+00, x) : copysign(r, x);
}

// acl_atan_fast with the range reduction read from a table (`tab`, 5 rows
// of {a, b, c, d, hi, lo}: t = (a|x| + b) / (c|x| + d), atan = hi + ...):
// three LDS reads instead of four select chains, far fewer live registers.
// kAtanTab is the table's content; callers stage it in LDS.
__device__ constexpr double kAtanTab[5][6] = {
    {1.0, 0.0, 0.0, 1.0, 0.0, 0.0},
    {2.0, -1.0, 1.0, 2.0, 4.63647609000806093515e-01, 2.26987774529616870924e-17},
    {1.0, -1.0, 1.0, 1.0, 7.85398163397448278999e-01, 3.06161699786838301793e-17},
    {1.0, -1.5, 1.5, 1.0, 9.82793723247329054082e-01, 1.39033110312309984516e-17},
    {0.0, -1.0, 1.0, 0.0, 1.57079632679489655800e+00, 6.12323399573676603587e-17}};

// a * b + C for a compile-time constant C: the constant is built in a
// reserved SGPR pair by two s_mov_b32 (scalar issue, beside the vector
// stream) and used by one VOP3 v_fma_f64. Written out because the compiler
// turns Horner steps with a constant addend into v_mov_b64 + v_fmac_f64 (a
// vector copy per step) or keeps the constants live in SGPRs (spills).
template <unsigned long long C>
__device__ __forceinline__ double fma_k(double a, double b) {
  double r;
  asm("s_mov_b32 s98, %3\n\ts_mov_b32 s99, %4\n\tv_fma_f64 %0, %1, %2, s[98:99]"
      : "=v"(r)
      : "v"(a), "v"(b), "i"((unsigned)(C & 0xffffffffu)), "i"((unsigned)(C >> 32))
      : "s98", "s99");
  return r;
}
#define ACL_FMA_K(a, b, c) fma_k<__builtin_bit_cast(unsigned long long, (double)(c))>(a, b)

// a * C1 + C2 (two roundings) for compile-time constants, both built in the
// reserved SGPR pair: no VGPR holds a hoisted constant across a loop (the
// fused auction + control kernel runs its gain loop at the 80-VGPR limit).
template <unsigned long long C1, unsigned long long C2>
__device__ __forceinline__ double mul_add_k(double a) {
  double r;
  asm("s_mov_b32 s98, %2\n\ts_mov_b32 s99, %3\n\tv_mul_f64 %0, %1, s[98:99]\n\t"
      "s_mov_b32 s98, %4\n\ts_mov_b32 s99, %5\n\tv_add_f64 %0, %0, s[98:99]"
      : "=&v"(r)
      : "v"(a), "i"((unsigned)(C1 & 0xffffffffu)), "i"((unsigned)(C1 >> 32)),
        "i"((unsigned)(C2 & 0xffffffffu)), "i"((unsigned)(C2 >> 32))
      : "s98", "s99");
  return r;
}
#define ACL_MUL_ADD_K(a, c1, c2)                                       \
  mul_add_k<__builtin_bit_cast(unsigned long long, (double)(c1)),    \
            __builtin_bit_cast(unsigned long long, (double)(c2))>(a)

__device__ __forceinline__ double acl_atan_tab(double x, const double* tab) {
  const double ax = fabs(x);
  const int id = (ax >= 0.4375) + (ax >= 0.6875) + (ax >= 1.1875) + (ax >= 2.4375);
  const double* rw = tab + 6 * id;
  const double num = __builtin_fma(rw[0], ax, rw[1]);
  const double den = __builtin_fma(rw[2], ax, rw[3]);
  const double t = id ? div_nr(num, den) : ax;
  const double z = t * t, w = z * z;
  // fdlibm's coefficients, Horner in w
  double p1 = ACL_FMA_K(w, 1.62858201153657823623e-02, 4.97687799461593236017e-02);
  p1 = ACL_FMA_K(w, p1, 6.66107313738753120669e-02);
  p1 = ACL_FMA_K(w, p1, 9.09088713343650656196e-02);
  p1 = ACL_FMA_K(w, p1, 1.42857142725034663711e-01);
  p1 = ACL_FMA_K(w, p1, 3.33333333333329318027e-01);
  double p2 = ACL_FMA_K(w, -3.65315727442169155270e-02, -5.83357013379057348645e-02);
  p2 = ACL_FMA_K(w, p2, -7.69187620504482999495e-02);
  p2 = ACL_FMA_K(w, p2, -1.11111104054623557880e-01);
  p2 = ACL_FMA_K(w, p2, -1.99999999998764832476e-01);
  const double s1 = z * p1;
  const double s2 = w * p2;
  const double r = id ? rw[4] - (__builtin_fma(t, s1 + s2, -rw[5]) - t)
                      : __builtin_fma(-t, s1 + s2, t);
  return (ax == __builtin_inf()) ? copysign(1.57079632679489655800e+00, x) : copysign(r, x);
}

// Square root with one Goldschmidt step from v_rsq_f64 (relative error
// ~2^-46): the distances of the control law's gated terms, where the parity
// bar is 1e-5 relative on u. sqrt(negative) and NaN give NaN, +-0 and +inf
// themselves, as std::sqrt.
__device__ __forceinline__ double sqrt_nr1(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  const double g = x * y, h = 0.5 * y;
  const double r = __builtin_fma(-g, h, 0.5);
  const double s = __builtin_fma(g, r, g);
  return (x == 0.0 || __builtin_isinf(x)) ? x : s;
}

// Rows k = 0..16 of {na, nb, da, db, a_k} for acl_atan_k32:
// atan(|x|) = a_k + atan(t), t = (na |x| + nb) / (da |x| + db), i.e.
// t = (|x| - c_k) / (1 + c_k |x|) with c_k = tan(k pi / 32), a_k = atan(c_k);
// k = 16: t = -1 / |x|, a = pi / 2. Callers stage it in LDS.
__device__ constexpr double kAtan32Tab[17][5] = {
    {1.0, 0.0, 0.0, 1.0, 0.0},
    {1.0, -0.09849140335716425, 0.09849140335716425, 1.0, 0.09817477042468103},
    {1.0, -0.198912367379658, 0.198912367379658, 1.0, 0.19634954084936207},
    {1.0, -0.3033466836073424, 0.3033466836073424, 1.0, 0.2945243112740431},
    {1.0, -0.41421356237309503, 0.41421356237309503, 1.0, 0.39269908169872414},
    {1.0, -0.5345111359507916, 0.5345111359507916, 1.0, 0.4908738521234052},
    {1.0, -0.6681786379192989, 0.6681786379192989, 1.0, 0.5890486225480862},
    {1.0, -0.8206787908286602, 0.8206787908286602, 1.0, 0.6872233929727672},
    {1.0, -0.9999999999999999, 0.9999999999999999, 1.0, 0.7853981633974483},
    {1.0, -1.2185035255879764, 1.2185035255879764, 1.0, 0.8835729338221293},
    {1.0, -1.496605762665489, 1.496605762665489, 1.0, 0.9817477042468103},
    {1.0, -1.8708684117893888, 1.8708684117893888, 1.0, 1.0799224746714913},
    {1.0, -2.414213562373095, 2.414213562373095, 1.0, 1.1780972450961724},
    {1.0, -3.296558208938321, 3.296558208938321, 1.0, 1.2762720155208536},
    {1.0, -5.027339492125846, 5.027339492125846, 1.0, 1.3744467859455345},
    {1.0, -10.153170387608842, 10.153170387608842, 1.0, 1.4726215563702154},
    {0.0, -1.0, 1.0, 0.0, 1.5707963267948966}};

// atan for the control law's gated terms (parity bar 1e-5 relative on u). An
// fp32 estimate of atan(|x|) (pi/4 y - y (y - 1)(0.2447 + 0.0663 y) on
// y = min(|x|, 1/|x|), |error| < 2e-3 rad) picks the nearest table point, so
// |t| <= tan(pi/64 + 2e-3) < 0.052, and atan(t) = t + t z (-1/3 + z/5 - z^2/7
// + z^3/9), z = t^2, is within z^5 / 11 < 1.3e-14 relative. One reciprocal
// with one Newton step for the quotient.
__device__ __forceinline__ double acl_atan_k32(double x, const double* tab) {
  const double ax = fabs(x);
  const float xf = (float)ax;
  const bool big = xf > 1.0f;
  const float yf = big ? __builtin_amdgcn_rcpf(xf) : xf;
  const float t0 = yf * (0.78539816f - (yf - 1.0f) * (0.2447f + 0.0663f * yf));
  const float th = big ? 1.57079633f - t0 : t0;
  int k = (int)(th * 10.18591636f + 0.5f);  // round(th * 32 / pi)
  k = k < 0 ? 0 : (k > 16 ? 16 : k);
  const double* rw = tab + 5 * k;
  const double num = __builtin_fma(rw[0], ax, rw[1]);
  const double den = __builtin_fma(rw[2], ax, rw[3]);
  double r = __builtin_amdgcn_rcp(den);
  r = __builtin_fma(__builtin_fma(-den, r, 1.0), r, r);
  const double t = num * r;
  const double z = t * t;
  double p = ACL_MUL_ADD_K(z, 1.0 / 9.0, -1.0 / 7.0);
  p = ACL_FMA_K(z, p, 1.0 / 5.0);
  p = ACL_FMA_K(z, p, -1.0 / 3.0);
  const double res = rw[4] + __builtin_fma(t * z, p, t);
  return (ax == __builtin_inf()) ? copysign(1.57079632679489655800e+00, x) : copysign(res, x);
}

// Rows k = 0..33 of {na, nb, da, db, a_k} for acl_atan_b: row 0 (|x| <
// 2^-4) is atan itself (c = 0); rows 1..32 split [2^-4, 2^4) into binades of
// four linear steps, c_k = tan of the midpoint of the step's atan range
// (a_k = atan(c_k)), t = (|x| - c_k) / (1 + c_k |x|); row 33 (|x| >= 16):
// t = -1 / |x|, a = pi / 2. |t| <= 0.0625 everywhere. Callers stage it in LDS.
__device__ constexpr double kAtanBTab[34][5] = {
    {1.0, 0.0, 0.0, 1.0, 0.0},
    {1.0, -0.07030822983596466, 0.07030822983596466, 1.0, 0.07019272191374983},
    {1.0, -0.08593229355760532, 0.08593229355760532, 1.0, 0.08572170749506589},
    {1.0, -0.10155636477210132, 0.10155636477210132, 1.0, 0.10120936907422763},
    {1.0, -0.11718044475643763, 0.11718044475643763, 1.0, 0.11664847576831361},
    {1.0, -0.14059134139479385, 0.14059134139479385, 1.0, 0.13967586823535122},
    {1.0, -0.1718342517380426, 0.1718342517380426, 1.0, 0.17017234595981787},
    {1.0, -0.20307738469612643, 0.20307738469612643, 1.0, 0.2003528248467164},
    {1.0, -0.2343207709802973, 0.2343207709802973, 1.0, 0.2301681814123011},
    {1.0, -0.28099568840305256, 0.28099568840305256, 1.0, 0.27393176575091777},
    {1.0, -0.34345001598898495, 0.34345001598898495, 1.0, 0.3308277693227718},
    {1.0, -0.40590971677575227, 0.40590971677575227, 1.0, 0.3855905559339798},
    {1.0, -0.4683749459844424, 0.4683749459844424, 1.0, 0.4380290252990967},
    {1.0, -0.560834617207166, 0.560834617207166, 1.0, 0.5111234621721843},
    {1.0, -0.6856796740973412, 0.6856796740973412, 1.0, 0.6010502120684234},
    {1.0, -0.8105909435321778, 0.8105909435321778, 1.0, 0.6811655542074544},
    {1.0, -0.9355530918915272, 0.9355530918915272, 1.0, 0.7521140815095364},
    {1.0, -1.1172650153486017, 1.1172650153486017, 1.0, 0.8407267739843961},
    {1.0, -1.3675814891468359, 1.3675814891468359, 1.0, 0.9394245539093364},
    {1.0, -1.618033988749895, 1.618033988749895, 1.0, 1.0172219678978514},
    {1.0, -1.8685170918213303, 1.8685170918213303, 1.0, 1.0793994651712322},
    {1.0, -2.2268438420880323, 2.2268438420880323, 1.0, 1.148719333738311},
    {1.0, -2.729944215084218, 2.729944215084218, 1.0, 1.219667861040393},
    {1.0, -3.232440682034051, 3.232440682034051, 1.0, 1.2707712200940198},
    {1.0, -3.734444135973819, 3.734444135973819, 1.0, 1.309157165728909},
    {1.0, -4.44708844906985, 4.44708844906985, 1.0, 1.3496092153065242},
    {1.0, -5.4560113489583335, 5.4560113489583335, 1.0, 1.3895242081626429},
    {1.0, -6.462432795016398, 6.462432795016398, 1.0, 1.4172734607855013},
    {1.0, -7.467251416997126, 7.467251416997126, 1.0, 1.437670302219434},
    {1.0, -8.890260421989915, 8.890260421989915, 1.0, 1.4587845032759348},
    {1.0, -10.909842172583009, 10.909842172583009, 1.0, 1.479391384605095},
    {1.0, -12.923532073277041, 12.923532073277041, 1.0, 1.4935719784580308},
    {1.0, -14.93362962377707, 14.93362962377707, 1.0, 1.5039331894042727},
    {0.0, -1.0, 1.0, 0.0, 1.5707963267948966},
};

// atan for the control law's gated terms (parity bar 1e-5 relative on u):
// the row is picked by the float bits of |x| -- exponent and the top two
// mantissa bits, (bits >> 21) - (123 << 2) + 1 clamped to [0, 33], four
// integer instructions -- and atan(t) = t + t z (-1/3 + z/5 - z^2/7 + z^3/9
// - z^4/11), z = t^2, is within 4e-16 relative on |t| <= 0.0625
// (tests/test_fastmath.py). One reciprocal with one Newton step. The row's
// five coefficients are five LDS reads: a 16-byte {c, a} row with the last
// row selected measured no faster and cost the vector ALU -- which bounds the
// fused kernel -- four selects per call (profiles/r6_ab_atan/).
__device__ __forceinline__ double acl_atan_b(double x, const double* tab) {
  const double ax = fabs(x);
  int k = (int)(__float_as_uint((float)ax) >> 21) - (123 << 2) + 1;
  k = k < 0 ? 0 : (k > 33 ? 33 : k);
  const double* rw = tab + 5 * k;
  const double num = __builtin_fma(rw[0], ax, rw[1]);
  const double den = __builtin_fma(rw[2], ax, rw[3]);
  double r = __builtin_amdgcn_rcp(den);
  r = __builtin_fma(__builtin_fma(-den, r, 1.0), r, r);
  const double t = num * r;
  const double z = t * t;
  double p = ACL_MUL_ADD_K(z, -1.0 / 11.0, 1.0 / 9.0);
  p = ACL_FMA_K(z, p, -1.0 / 7.0);
  p = ACL_FMA_K(z, p, 1.0 / 5.0);
  p = ACL_FMA_K(z, p, -1.0 / 3.0);
  const double res = rw[4] + __builtin_fma(t * z, p, t);
  return (ax == __builtin_inf()) ? copysign(1.57079632679489655800e+00, x) : copysign(res, x);
}

// getPrice (auctioneer.cpp:546-549) from the squared distance x:
// (float)(1.0 / (sqrt(x) + 1e-8)) with IEEE sqrt and division, bit for bit.
// The fast path computes y = 1 / (sqrt(x) + 1e-8) with sqrt_nr and div_nr
// (a few ulp of the exact double in all) and rounds it to float; that float
// is the exact one unless a float rounding boundary (a midpoint between two
// floats) lies within the error: the 29 mantissa bits the float drops are
// then within 1024 ulp of their midpoint 2^28, and those lanes (about 4e-6
// of them) -- and every x outside [1e-200, 1e60] (zero, subnormal results,
// float underflow, inf, NaN) -- take the IEEE expression. `tests/
// test_gpu_prices.py` sweeps it against the IEEE expression on the GPU.
//
// y = 1 / (s + 1e-8) = r / (1 + d) with r = 1/sqrt(x), d = 1e-8 r: r from the
// hardware reciprocal square root and two Newton steps (each squares the
// relative error, then a few ulp of rounding), y = r (1 - d + d^2) -- the
// truncated d^3 is below 1e-15 relative for x > 1e-6 (distances above 1 mm;
// smaller x take the IEEE expression): one transcendental and eleven
// arithmetic instructions instead of a square root and a quotient by Newton
// steps (two transcendentals, seventeen).
#ifndef ACL_PRICE_RSQ
#define ACL_PRICE_RSQ 1
#endif
__device__ __forceinline__ float acl_price(double x) {
#if ACL_PRICE_RSQ
  double r = __builtin_amdgcn_rsq(x);
  double t = x * r;
  double e = __builtin_fma(-t, r, 1.0);
  r = __builtin_fma(0.5 * r, e, r);
  t = x * r;
  e = __builtin_fma(-t, r, 1.0);
  r = __builtin_fma(0.5 * r, e, r);
  const double d = 1e-8 * r;
  const double y = __builtin_fma(r, __builtin_fma(d, d, -d), r);
  const double lo = 1e-6;
#else
  const double y = div_nr(1.0, sqrt_nr(x) + 1e-8);
  const double lo = 1e-200;
#endif
  const unsigned r29 = (unsigned)((unsigned long long)__double_as_longlong(y) & ((1ull << 29) - 1ull));
  const bool fast = x > lo && x < 1e60 && (r29 - (1u << 28) + 1024u) > 2048u;
  float c = (float)y;
  if (!fast) c = (float)(1.0 / (sqrt(x) + 1e-8));
  return c;
}

__device__ __forceinline__ double wrap_to_pi(double a) {  // utils.h:275-280
  if (a > kPi) return a - 2 * kPi;
  if (a < -kPi) return a + 2 * kPi;
  return a;
}

}  // namespace acl_amd

namespace acl_amd {

// ---- round work by ticket (the auction kernels' column updates and re-selects)
// the k-th set bit (k < popcount) of the NW-word mask m (wave-uniform)
__device__ __forceinline__ int kth_bit(const unsigned long long* m, int NW, int k) {
  for (int w = 0; w < NW; ++w) {
    unsigned long long x = m[w];
    const int pc = __popcll(x);
    if (k < pc) {
      for (int q = 0; q < k; ++q) x &= x - 1;
      return 64 * w + __ffsll((long long)x) - 1;
    }
    k -= pc;
  }
  return -1;
}

// a ticket from the workgroup's counter at misc[slot] (wave-uniform)
__device__ __forceinline__ int wave_ticket(int* misc, int slot, int lane) {
  int t = 0;
  if (lane == 0) t = atomicAdd(&misc[slot], 1);
  return __builtin_amdgcn_readfirstlane(t);
}

// ---- decision margin (include/aclswarm_amd.h, acl_swarm_status_t::margin) --
// A thread tracks the compared f32 pair (hi, lo), hi >= lo >= 0, with the
// largest ratio lo / hi: products of two floats are exact in double, so the
// ranking is exact and order-independent; a tie (lo == hi) is ratio 1. The
// oracle (oracle/aclswarm_oracle.c, orc_margin_track) is the same function.
struct MarginPair {
  float hi, lo;
};

__device__ __forceinline__ void margin_init(MarginPair& m) {
  m.hi = 1.0f;
  m.lo = 0.0f;
}

__device__ __forceinline__ void margin_track(MarginPair& m, float hi, float lo) {
  if (!(lo < hi)) {
    if (lo == hi) {
      m.hi = 1.0f;
      m.lo = 1.0f;
    }
    return;  // NaN: the swarm is NONFINITE (margin 0)
  }
  if ((double)lo * (double)m.hi > (double)m.lo * (double)hi) {
    m.hi = hi;
    m.lo = lo;
  }
}

// this lane's bit of a wave lane mask (a per-lane predicate, no VALU)
__device__ __forceinline__ bool lanebit_u64(unsigned long long m) {
  return __builtin_amdgcn_inverse_ballot_w64(m);
}

// a per-lane flag held as a VGPR integer (0 or 1), combined with bitwise
// vector operations (the compiler would keep a divergent bool as an SGPR
// lane mask combined by scalar instructions; the auction kernels are bound
// by the CU's scalar pipe)
__device__ __forceinline__ unsigned vflag(bool x) {
  unsigned v = x ? 1u : 0u;
  asm volatile("" : "+v"(v));
  return v;
}

// margin_track of a per-lane pair where `act`, branch-free: the
// kernel is bound by the CU's scalar pipe, and a divergent branch costs three
// scalar instructions (exec save, branch, restore) where selects cost none
__device__ __forceinline__ void margin_track_sel(MarginPair& m, float hi, float lo, bool act) {
  const bool eq = act && lo == hi;
  const bool up = act && lo < hi && (double)lo * (double)m.hi > (double)m.lo * (double)hi;
  m.hi = eq ? 1.0f : (up ? hi : m.hi);
  m.lo = eq ? 1.0f : (up ? lo : m.lo);
}

// gap of a tracked pair: (hi - lo) / hi in double (hi - lo exact there), 1
// when lo < 2^-28 hi; monotone in the ratio, so min over gaps = gap of the
// max-ratio pair
__device__ __forceinline__ double margin_gap(const MarginPair& m) {
  const double hi = m.hi, lo = m.lo;
  if (lo * 268435456.0 < hi) return 1.0;
  return (hi - lo) / hi;
}

// Decision gap of the alignment's determinant-sign and rank tests
// (Eigen::umeyama 3.3.x, auctioneer.cpp:397), as orc_umeyama2_gap.
__device__ __forceinline__ double align_gap(const double S[4], double det, const double sv[2]) {
  const double den = fabs(S[0] * S[3]) + fabs(S[2] * S[1]);
  double g = (den > 0.0) ? fabs(det) / den : 0.0;
  if (!(g <= 1.0)) g = (g > 1.0) ? 1.0 : 0.0;
  const double th = fabs(sv[0]) * 1e-12, a = fabs(sv[1]);
  const double mx = (a > th) ? a : th;
  const double gr = (mx > 0.0) ? fabs(a - th) / mx : 0.0;
  return (gr < g) ? gr : g;
}

// non-negative doubles order like their bit patterns: block minimum through
// one LDS word (initialised to 1.0)
__device__ __forceinline__ void block_min_gap(unsigned long long* word, double g) {
  const unsigned long long bits = (unsigned long long)__double_as_longlong(g);
  const unsigned long long m = ~wave_max_u64(~bits);  // wave minimum
  if ((threadIdx.x & 63) == 0) atomicMin(word, m);
}

}  // namespace acl_amd
