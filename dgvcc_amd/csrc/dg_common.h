// Shared device helpers for the DGVCC MI355X (gfx950) kernels.
// Layout convention for every activation tensor: NHWC with an explicit pixel
// stride `ld` (elements between consecutive pixels), so a channel slice of a
// wider buffer (the decoder's concatenations) is addressed in place.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <stdint.h>
#include <type_traits>
#include "../../include/dgvcc.h"

typedef __bf16 bf16;
typedef _Float16 f16;  // fp16 storage mode (configs/qnrf_final.yml): same 16-bit layouts as bf16
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
#define DG_IS16(dt) ((dt) == DG_BF16 || (dt) == DG_F16)
template <typename T> struct Is16 { static constexpr bool value = false; };
template <> struct Is16<bf16> { static constexpr bool value = true; };
template <> struct Is16<f16> { static constexpr bool value = true; };
typedef short s8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));  // native 16-B vector (SROA-friendly, unlike HIP's uint4 struct)

#define DG_LDS __attribute__((address_space(3)))

#define DG_CHECK_LAUNCH()                                  \
  do {                                                     \
    hipError_t e_ = hipGetLastError();                     \
    if (e_ != hipSuccess) return DG_ERR_HIP;               \
  } while (0)

#define DG_REQUIRE(cond)                                   \
  do {                                                     \
    if (!(cond)) return DG_ERR_INVALID;                    \
  } while (0)

#define DG_SUPPORTED(cond)                                 \
  do {                                                     \
    if (!(cond)) return DG_ERR_UNSUPPORTED;                \
  } while (0)

__device__ __forceinline__ float bf2f(unsigned short u) { return __uint_as_float(((unsigned)u) << 16); }
__device__ __forceinline__ unsigned short f2bf(float x) { return __builtin_bit_cast(unsigned short, (bf16)x); }

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
__device__ __forceinline__ float to_f(f16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }
template <> __device__ __forceinline__ f16 from_f<f16>(float x) { return (f16)x; }
// x rounded to the storage type T and back (the value a later pass will read)
template <typename T> __device__ __forceinline__ float round_to(float x) { return to_f(from_f<T>(x)); }
__device__ __forceinline__ float h2f(unsigned short u) { return (float)__builtin_bit_cast(f16, u); }
__device__ __forceinline__ unsigned short f2h(float x) { return __builtin_bit_cast(unsigned short, (f16)x); }
// 16-bit payload <-> float for a storage type H (bf16 or f16)
template <typename H> __device__ __forceinline__ float u16_to_f(unsigned short u) {
  if constexpr (std::is_same<H, bf16>::value) return bf2f(u); else return h2f(u);
}
template <typename H> __device__ __forceinline__ unsigned short f_to_u16(float x) {
  if constexpr (std::is_same<H, bf16>::value) return f2bf(x); else return f2h(x);
}
// v_mfma_f32_16x16x32_{bf16,f16}: the same operand/accumulator layouts (cdna_hip_programming.md §3)
template <typename H> __device__ __forceinline__ f4v mfma16x16x32(const s8v& a, const s8v& b, const f4v& c) {
  if constexpr (std::is_same<H, bf16>::value)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, a), __builtin_bit_cast(h8v, b), c, 0, 0,
                                                    0);
}

typedef unsigned u2v __attribute__((ext_vector_type(2)));

// 4-element vector load/store through float registers.
__device__ __forceinline__ void ld4(const float* p, float v[4]) {
  f4v t = *(const f4v*)p;
  v[0] = t[0]; v[1] = t[1]; v[2] = t[2]; v[3] = t[3];
}
__device__ __forceinline__ void ld4(const bf16* p, float v[4]) {
  u2v t = *(const u2v*)p;
  v[0] = __uint_as_float(t[0] << 16); v[1] = __uint_as_float(t[0] & 0xffff0000u);
  v[2] = __uint_as_float(t[1] << 16); v[3] = __uint_as_float(t[1] & 0xffff0000u);
}
__device__ __forceinline__ void ld4(const f16* p, float v[4]) {
  u2v t = *(const u2v*)p;
  v[0] = h2f((unsigned short)(t[0] & 0xffffu)); v[1] = h2f((unsigned short)(t[0] >> 16));
  v[2] = h2f((unsigned short)(t[1] & 0xffffu)); v[3] = h2f((unsigned short)(t[1] >> 16));
}
__device__ __forceinline__ unsigned pack_h2(float lo, float hi) {
  return (unsigned)f2h(lo) | ((unsigned)f2h(hi) << 16);
}
__device__ __forceinline__ void st4(f16* p, const float v[4]) {
  *(u2v*)p = u2v{pack_h2(v[0], v[1]), pack_h2(v[2], v[3])};
}
__device__ __forceinline__ void st4(float* p, const float v[4]) { *(f4v*)p = f4v{v[0], v[1], v[2], v[3]}; }
__device__ __forceinline__ unsigned pack_bf2(float lo, float hi) {
  return (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
}
__device__ __forceinline__ void st4(bf16* p, const float v[4]) {
  *(u2v*)p = u2v{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
}

// 16-byte vector = VEC elements (4 f32 or 8 bf16).
template <typename T> struct VecT { static constexpr int N = 16 / sizeof(T); };
__device__ __forceinline__ void ldv(const float* p, float v[4]) { ld4(p, v); }
__device__ __forceinline__ void ldv(const bf16* p, float v[8]) {
  u4v t = *(const u4v*)p;
#pragma unroll
  for (int i = 0; i < 4; ++i) { v[2 * i] = __uint_as_float(t[i] << 16); v[2 * i + 1] = __uint_as_float(t[i] & 0xffff0000u); }
}
__device__ __forceinline__ void ldv(const f16* p, float v[8]) {
  u4v t = *(const u4v*)p;
#pragma unroll
  for (int i = 0; i < 4; ++i) { v[2 * i] = h2f((unsigned short)(t[i] & 0xffffu)); v[2 * i + 1] = h2f((unsigned short)(t[i] >> 16)); }
}
__device__ __forceinline__ void stv(f16* p, const float v[8]) {
  *(u4v*)p = u4v{pack_h2(v[0], v[1]), pack_h2(v[2], v[3]), pack_h2(v[4], v[5]), pack_h2(v[6], v[7])};
}
__device__ __forceinline__ void stv(float* p, const float v[4]) { st4(p, v); }
__device__ __forceinline__ void stv(bf16* p, const float v[8]) {
  *(u4v*)p = u4v{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7])};
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): consecutive logical tiles land on the same XCD so neighbouring
// tiles that share operand panels hit the same L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

static inline int dg_cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// Words of an f32 output's operand-maxima buffer: 1 + C (the tensor's word, then one per channel:
// OutMax), rounded up to a multiple of 4 so the zeroing below is one 16-byte-aligned fill (a 4(1 + C)-byte
// memset ran as two fill dispatches); 16-bit outputs use word 0 alone.
__host__ __device__ inline size_t dg_amax_words(int C) { return ((size_t)C + 4) & ~(size_t)3; }
// Zero a producer's operand-maxima buffer before its launch (may be NULL).  DG_ERR_INVALID when an f32
// output has more channels than the per-channel fold handles.
static inline int dg_zero_amax(float* amax, int dtype, int C, hipStream_t st) {
  if (!amax) return DG_OK;
  if (dtype == DG_F32 && C > 2048) return DG_ERR_INVALID;  // DG_CAMAX_C
  return hipMemsetAsync(amax, 0, (dtype == DG_F32 ? dg_amax_words(C) : 1) * 4, st) == hipSuccess ? DG_OK : DG_ERR_HIP;
}

// ---------------------------------------------------------------------------
// f32 arithmetic on the bf16 matrix cores ("3-way split", DG_F32 with
// dg_set_f32_math(1)).  Each f32 x is cut EXACTLY into three bf16 parts, x = h0 + h1 + h2
// (x - h0 spans <= 16 significant bits and its remainder <= 8, so h2 is exact in bf16; the
// identity-filter test checks it bit for bit on every kernel path); a product x*y is then
// sum_{i+j<=2} xi*yj, six v_mfma_f32_16x16x32_bf16 per 16x16x32 block with f32 accumulation,
// products of bf16 being exact in f32.  Six bf16 MFMAs (16 cycles each) replace eight
// v_mfma_f32_16x16x4_f32 (32 cycles each) per 32-deep K block.  Two rounding rules for the
// parts, each where it measured better (tests/test_kernels_gpu.py):
//  * truncation (split3_8 / split3_4 / split_weight_kernel: forward and dgrad, K <= 4608):
//    every part carries its operand's sign.  The rounding of the two photometric views of a
//    final-mode step then stays correlated through the network, so the consistency loss
//    between them (a mean of squared differences of near-equal softmaxes, ~1e-8) comes out
//    at 5e-7 relative to float64, against 1.8e-4 with nearest parts and 8.7e-5 on the exact
//    f32 MFMA; the one-sided dropped terms (|x1*y2|, |x2*y1| < 2^-21 |x*y|, typically ~2^-22
//    of sum |x*y|) stay below the f32 accumulation error of these sums (same-sign K = 4608:
//    4.2e-6 against 5.0e-6 exact).
//  * round-to-nearest-even (split3_8_rn / split3_4_rn, one v_cvt_pk_bf16_f32 per pair and
//    level: weight gradients, reductions over up to 786k pixels): with truncation, same-sign
//    operands (post-ReLU x, positive dy) make the small products x2*y0, x1*y1, x0*y2 (~2^-16
//    |x*y| each) all push one way, and once the accumulator of a long reduction is ~2^12
//    products large a 32-deep block of them falls under its half-ulp and is rounded away in
//    the same direction every block: 1.1e-5 relative on the 786k-pixel wgrad, 10x the exact
//    MFMA.  Nearest parts are sign-symmetric (|h1| <= 2^-8 |x|, |h2| <= 2^-16 |x|): 3.7e-7.
// ---------------------------------------------------------------------------
typedef __bf16 dg_bf16x2 __attribute__((ext_vector_type(2)));
typedef float dg_f32x2 __attribute__((ext_vector_type(2)));
// RN-even bf16 pair (lo = a, hi = b): one v_cvt_pk_bf16_f32
__device__ __forceinline__ unsigned cvt_pk_bf16(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(dg_f32x2{a, b}, dg_bf16x2));
}
// one nearest split level of a pair: the packed parts, and the exact f32 remainders
__device__ __forceinline__ unsigned split_level2(float a, float b, float& ra, float& rb) {
  const unsigned p = cvt_pk_bf16(a, b);
  ra = a - __uint_as_float(p << 16);
  rb = b - __uint_as_float(p & 0xffff0000u);
  return p;
}
// the parts of a pair of f32 (bit patterns a, b), packed lo = a, hi = b
// (the remainders are formed as float pairs: one v_pk_add_f32 per level and pair)
typedef unsigned dg_u32x2 __attribute__((ext_vector_type(2)));
template <bool RN>
__device__ __forceinline__ void split3_pair(unsigned a, unsigned b, unsigned& p0, unsigned& p1, unsigned& p2) {
  if constexpr (RN) {
    float ra, rb, sa, sb;
    p0 = split_level2(__uint_as_float(a), __uint_as_float(b), ra, rb);
    p1 = split_level2(ra, rb, sa, sb);
    p2 = cvt_pk_bf16(sa, sb);  // exact
  } else {
    const dg_u32x2 x = {a, b};
    p0 = __builtin_amdgcn_perm(b, a, 0x07060302u);  // (a >> 16) | (b & 0xffff0000)
    const dg_f32x2 r = __builtin_bit_cast(dg_f32x2, x) - __builtin_bit_cast(dg_f32x2, x & 0xffff0000u);
    const dg_u32x2 ur = __builtin_bit_cast(dg_u32x2, r);
    p1 = __builtin_amdgcn_perm(ur.y, ur.x, 0x07060302u);
    const dg_f32x2 q = r - __builtin_bit_cast(dg_f32x2, ur & 0xffff0000u);
    const dg_u32x2 uq = __builtin_bit_cast(dg_u32x2, q);
    p2 = __builtin_amdgcn_perm(uq.y, uq.x, 0x07060302u);
  }
}
// 8 f32 (x0[0..3], x1[0..3]) -> bf16 parts h0/h1/h2, element k of each part = float k
template <bool RN = false>
__device__ __forceinline__ void split3_8t(const u4v& x0, const u4v& x1, s8v& h0, s8v& h1, s8v& h2) {
  u4v p0, p1, p2;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const unsigned a = k < 2 ? x0[2 * k] : x1[2 * k - 4];
    const unsigned b = k < 2 ? x0[2 * k + 1] : x1[2 * k - 3];
    unsigned q0, q1, q2;
    split3_pair<RN>(a, b, q0, q1, q2);
    p0[k] = q0;
    p1[k] = q1;
    p2[k] = q2;
  }
  h0 = __builtin_bit_cast(s8v, p0);
  h1 = __builtin_bit_cast(s8v, p1);
  h2 = __builtin_bit_cast(s8v, p2);
}
__device__ __forceinline__ void split3_8(const u4v& x0, const u4v& x1, s8v& h0, s8v& h1, s8v& h2) {
  split3_8t<false>(x0, x1, h0, h1, h2);
}
__device__ __forceinline__ void split3_8_rn(const u4v& x0, const u4v& x1, s8v& h0, s8v& h1, s8v& h2) {
  split3_8t<true>(x0, x1, h0, h1, h2);
}
// the six products of one block, smallest first (all into the same f32 accumulator)
__device__ __forceinline__ f4v mfma_x6(const s8v& a0, const s8v& a1, const s8v& a2, const s8v& b0, const s8v& b1,
                                       const s8v& b2, f4v c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, b0, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b2, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b0, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b1, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, c, 0, 0, 0);
  return c;
}

// 4 f32 -> the bf16 parts of each (element k of part p = part p of x[k])
template <bool RN = false>
__device__ __forceinline__ void split3_4t(const u4v& x, u2v& h0, u2v& h1, u2v& h2) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    unsigned p0, p1, p2;
    split3_pair<RN>(x[2 * k], x[2 * k + 1], p0, p1, p2);
    h0[k] = p0;
    h1[k] = p1;
    h2[k] = p2;
  }
}
__device__ __forceinline__ void split3_4(const u4v& x, u2v& h0, u2v& h1, u2v& h2) { split3_4t<false>(x, h0, h1, h2); }
__device__ __forceinline__ void split3_4_rn(const u4v& x, u2v& h0, u2v& h1, u2v& h2) { split3_4t<true>(x, h0, h1, h2); }

// ---------------------------------------------------------------------------
// f32 arithmetic on the f16 matrix cores ("f16 x3", DG_F32 with dg_set_f32_math(2)): each
// f32 operand, scaled by a power of two s into f16 range (|x*s| < 2^14; s per filter row, per
// tensor for the pixel operand), is cut into two f16 parts by nearest rounding,
// x*s = hi + lo + r with |lo| <= 2^-11 |x*s| and |r| <= 2^-23 |x*s|; a product is then
// hi*hi + hi*lo + lo*hi, three v_mfma_f32_16x16x32_f16 per 16x16x32 block with f32
// accumulation (f16 products are exact in f32), and the result is scaled back by the exact
// 1/(s_a*s_b).  Dropped per product: lo*lo (<= 2^-22) and the parts' rounding (<= 2^-22),
// two-sided.  Values below 2^-3 after scaling get a subnormal lo part: absolute error
// <= 2^-25 in scaled units, i.e. <= 2^-39 of the operand's largest element.  Three 16-cycle
// MFMAs per 32-deep block instead of the 3-way bf16 split's six.
// ---------------------------------------------------------------------------
typedef _Float16 dg_f16x2 __attribute__((ext_vector_type(2)));
// power-of-two scale taking |x| <= amax below 2^14 (amax = m 2^e, m in [0.5, 1) -> 2^(14-e))
__device__ __forceinline__ int h16_exp(float amax) {
  if (!(amax > 0.f) || !(amax <= 3.4e38f)) return 0;
  int e;
  (void)frexpf(amax, &e);
  return max(-100, min(100, 14 - e));
}
// the f16 parts of a pair (lo = a, hi = b in each packed dword) of x * s
__device__ __forceinline__ void split2h_pair(float a, float b, float s, unsigned& ph, unsigned& pl) {
  const dg_f32x2 v = dg_f32x2{a, b} * s;
  const dg_f16x2 h = __builtin_convertvector(v, dg_f16x2);
  const dg_f32x2 r = v - __builtin_convertvector(h, dg_f32x2);
  ph = __builtin_bit_cast(unsigned, h);
  pl = __builtin_bit_cast(unsigned, __builtin_convertvector(r, dg_f16x2));
}
// 8 f32 (x0[0..3], x1[0..3]) -> f16 parts hi / lo of x * s, element k of each part = float k
__device__ __forceinline__ void split2h_8(const u4v& x0, const u4v& x1, float s, s8v& hi, s8v& lo) {
  u4v ph, pl;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const unsigned a = k < 2 ? x0[2 * k] : x1[2 * k - 4];
    const unsigned b = k < 2 ? x0[2 * k + 1] : x1[2 * k - 3];
    unsigned qh, ql;
    split2h_pair(__uint_as_float(a), __uint_as_float(b), s, qh, ql);
    ph[k] = qh;
    pl[k] = ql;
  }
  hi = __builtin_bit_cast(s8v, ph);
  lo = __builtin_bit_cast(s8v, pl);
}
// the three products of one block, smallest first
__device__ __forceinline__ f4v mfma_h3(const s8v& ah, const s8v& al, const s8v& bh, const s8v& bl, f4v c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, al), __builtin_bit_cast(h8v, bh), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, ah), __builtin_bit_cast(h8v, bl), c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, ah), __builtin_bit_cast(h8v, bh), c, 0, 0, 0);
  return c;
}
// 4 f32 -> the f16 parts of x * s (element k of part p = part p of x[k] * s)
__device__ __forceinline__ void split2h_4(const u4v& x, float s, u2v& hi, u2v& lo) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    unsigned qh, ql;
    split2h_pair(__uint_as_float(x[2 * k]), __uint_as_float(x[2 * k + 1]), s, qh, ql);
    hi[k] = qh;
    lo[k] = ql;
  }
}
// the same with one scale per element (per-channel scales: x holds 4 consecutive channels); the
// packed multiply takes both factors from registers, so the instruction count is split2h_4's
__device__ __forceinline__ void split2h_4v(const u4v& x, const f4v& s, u2v& hi, u2v& lo) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const dg_f32x2 v = dg_f32x2{__uint_as_float(x[2 * k]), __uint_as_float(x[2 * k + 1])} *
                       dg_f32x2{s[2 * k], s[2 * k + 1]};
    const dg_f16x2 h = __builtin_convertvector(v, dg_f16x2);
    const dg_f32x2 r = v - __builtin_convertvector(h, dg_f32x2);
    hi[k] = __builtin_bit_cast(unsigned, h);
    lo[k] = __builtin_bit_cast(unsigned, __builtin_convertvector(r, dg_f16x2));
  }
}
// per-channel f16 x3 scales of 4 consecutive channels c .. c + 3 from an operand-maxima buffer (word 0
// the tensor's max, word 1 + c channel c's): the exponents, and the factors 2^e
__device__ __forceinline__ void chan_h16_scales(const unsigned* am, int c, int e[4], f4v& s) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    e[k] = h16_exp(__uint_as_float(am[1 + c + k]));
    s[k] = ldexpf(1.f, e[k]);
  }
}

// Fold a block's max r >= 0 into *out (f32 bits, an unsigned max; zeroed before the launch), skipping
// the atomic when *out already holds >= r: the word only grows, so a stale read costs at most an
// atomic that changes nothing.  Thousands of blocks each issuing an atomic on one address serialise
// (tools/bench_bn.py: 16384 blocks made a 0.07-ms f32 BN apply 0.20 ms).
// The check is a plain cached load (a relaxed atomic load compiled to a system-coherent one, a memory
// round trip per word that the per-channel folds paid C / blockDim times per block): a stale value is
// never larger than the word, so it can only add an atomic that changes nothing.
__device__ __forceinline__ void amax_fold(unsigned* out, float r) {
  const unsigned v = __float_as_uint(r);
  if (*(const unsigned*)out < v) atomicMax(out, v);
}

// max |v| of the values a block stored, folded into *out (amax_fold).  Every thread of the block
// calls it.
__device__ __forceinline__ void block_amax_commit(float m, float* out) {
  __shared__ float red[16];
  m = wave_max(m);
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = red[0];
    for (int i = 1; i < nw; ++i) r = fmaxf(r, red[i]);
    amax_fold((unsigned*)out, r);
  }
}

// Operand maxima of an f32 output with channels (the f16 x3 convs' scales): out is
// [1 + C] floats, out[0] = max |v| over the tensor and out[1 + c] = max |v| over channel c (c local to
// the slice the kernel wrote; zeroed before the launch).  m[e] is the calling thread's max over the
// channel c0 + e it stored (channel-stationary passes: every thread keeps its V channels); inactive
// threads pass zeros.  Channels are reduced in LDS first (one fold per channel per block), C <= DG_CAMAX_C.
// Every thread of the block calls it.
constexpr int DG_CAMAX_C = 2048;
template <int V>
__device__ __forceinline__ void block_camax_commit(const float (&m)[V], int c0, int C, float* out) {
  __shared__ unsigned cm[DG_CAMAX_C];
  for (int c = threadIdx.x; c < C; c += blockDim.x) cm[c] = 0u;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int e = 0; e < V; ++e) {
    if (m[e] > 0.f) atomicMax(&cm[c0 + e], __float_as_uint(m[e]));  // non-negative: bit order = value order
    t = fmaxf(t, m[e]);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const unsigned v = cm[c];
    if (v) amax_fold((unsigned*)out + 1 + c, __uint_as_float(v));
  }
  block_amax_commit(t, out);
}
// Block size of the f32 channel-stationary passes that fold per-channel maxima: 1024 threads, a
// quarter as many blocks as their 256-thread grids.  Every block folds its C channel words at its
// end and the blocks of a launch end together, so a launch issues ~blocks x C global atomics there:
// 1024 x 64 added 20-25 us to a 70-us BN apply on the 786432 x 64 shape, and the pooled and
// InstanceNorm passes' up-to-8192/16384-block grids paid more (tools/bench_bn.py,
// profiles/round6d/bn_wide.txt).  DGVCC_EW_NT=256 (read per launch): the 256-thread grids.  The
// 16-bit passes (one word per block) measured no different in the wide form (profiles/round6d:
// bf16 step 105.2 vs 105.1 ms) and keep 256 threads.
constexpr int DG_EW_WIDE = 1024;
inline bool dg_ew_wide(const float* amax, bool f32) {
  if (!amax || !f32) return false;
  const char* e = getenv("DGVCC_EW_NT");
  return !(e && e[0] == '2');
}

// A producer's running operand maxima (out_amax_commit's input): per channel for f32 outputs (the only
// ones an f16 x3 conv reads), one register for 16-bit ones, whose buffer holds the tensor's word alone
template <typename T, int V>
struct OutMax {
  static constexpr int K = sizeof(T) == 4 ? V : 1;
  float m[K];
  __device__ __forceinline__ OutMax() {
#pragma unroll
    for (int e = 0; e < K; ++e) m[e] = 0.f;
  }
  __device__ __forceinline__ void add(int e, float v) {
    float& r = m[K == 1 ? 0 : e];
    r = fmaxf(r, fabsf(v));
  }
  // every thread of the block calls it
  __device__ __forceinline__ void commit(int c0, int C, float* out) const {
    if constexpr (K == 1) block_amax_commit(m[0], out);
    else block_camax_commit<V>(m, c0, C, out);
  }
};
