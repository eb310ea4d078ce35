// Batch normalisation (training statistics) + ReLU (+ Dropout2d channel mask)
// for NHWC activations: replaces nn.BatchNorm2d/nn.ReLU of vgg16_bn.features
// (models/models.py:35-38) and ConvBlock(bn=True) (models/models.py:8-21).
//
// HBM-bound passes.  Statistics use per-channel shifted sums (shift = first
// pixel's value) reduced per block, then a double-precision finalize, so the
// variance does not cancel when |mean| >> std.
#include "dg_common.h"
#include <algorithm>
#include <cstdlib>

namespace {

constexpr int NT = 256;

inline int bn_nblk_cap() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DGVCC_BN_NBLK");
    v = e ? std::max(64, atoi(e)) : 1024;
  }
  return v;
}
inline int bn_nblk(int M) { return std::max(1, std::min(bn_nblk_cap(), dg_cdiv(M, 64))); }
// pooled BN backward partials: more, smaller blocks (each thread walks 2x2 windows; more
// loads in flight per CU)
inline int pool_nblk_cap() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DGVCC_POOL_NBLK");
    v = e ? atoi(e) : 2048;
    if (v < 1) v = 1;
  }
  return v;
}
inline int pool_nblk(long long Mp) { return (int)std::max(1LL, std::min((long long)pool_nblk_cap(), (Mp + 31) / 32)); }

template <typename T>
__global__ __launch_bounds__(NT) void bn_stats_partial(const T* __restrict__ z, long long ldz, int M, int C, int ppb,
                                                       float* __restrict__ part) {
  constexpr int V = 16 / (int)sizeof(T);
  __shared__ float sh[2][NT * V];
  const int tpp = C / V;
  const int rows = NT / tpp;
  const int tid = threadIdx.x;
  const int ch = tid % tpp, pl = tid / tpp;
  float s1[V], s2[V], K[V];
#pragma unroll
  for (int e = 0; e < V; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  const int p0 = blockIdx.x * ppb, p1 = min(M, p0 + ppb);
  if (pl < rows) {
    ldv(z + ch * V, K);
    for (int p = p0 + pl; p < p1; p += rows) {
      float v[V];
      ldv(z + (long long)p * ldz + ch * V, v);
#pragma unroll
      for (int e = 0; e < V; ++e) { const float d = v[e] - K[e]; s1[e] += d; s2[e] = fmaf(d, d, s2[e]); }
    }
#pragma unroll
    for (int e = 0; e < V; ++e) { sh[0][pl * C + ch * V + e] = s1[e]; sh[1][pl * C + ch * V + e] = s2[e]; }
  }
  __syncthreads();
  for (int c = tid; c < C; c += NT) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rows; ++r) { a += sh[0][r * C + c]; b += sh[1][r * C + c]; }
    part[(long long)blockIdx.x * 2 * C + c] = a;
    part[(long long)blockIdx.x * 2 * C + C + c] = b;
  }
}

// 16 channels per block, 16 lanes per channel striding over the block partials
// (independent loads, 4 in flight per lane), then an LDS combine in double.
// ROW = true: write this batch's (n, mean, M2) row [3][C] to save_mean instead (a SyncBatchNorm
// rank's local statistics, merged across ranks by dg_bn_part_finalize).
template <typename T, bool ROW = false>
__global__ __launch_bounds__(NT) void bn_stats_finalize(const T* __restrict__ z, const float* __restrict__ part,
                                                        int nblk, int M, int C, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float* running_mean,
                                                        float* running_var, float momentum, float eps,
                                                        float* save_mean, float* save_invstd, float* scale,
                                                        float* shift) {
  __shared__ double sh[2][16][17];
  const int cl = threadIdx.x & 15, r = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  double a = 0.0, b = 0.0;
  if (c < C) {
    int k = r;
    for (; k + 48 < nblk; k += 64) {
      float a4[4], b4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a4[u] = part[(long long)(k + 16 * u) * 2 * C + c];
        b4[u] = part[(long long)(k + 16 * u) * 2 * C + C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { a += a4[u]; b += b4[u]; }
    }
    for (; k < nblk; k += 16) { a += part[(long long)k * 2 * C + c]; b += part[(long long)k * 2 * C + C + c]; }
  }
  sh[0][r][cl] = a;
  sh[1][r][cl] = b;
  __syncthreads();
  if (r != 0 || c >= C) return;
  a = 0.0; b = 0.0;
  for (int q = 0; q < 16; ++q) { a += sh[0][q][cl]; b += sh[1][q][cl]; }
  const double K = (double)to_f(z[c]);
  const double ms = a / M;
  double var = b / M - ms * ms;
  if (var < 0) var = 0;
  const double mean = K + ms;
  if constexpr (ROW) {
    save_mean[c] = (float)M;
    save_mean[C + c] = (float)mean;
    save_mean[2 * C + c] = (float)(var * M);
    return;
  }
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  save_mean[c] = (float)mean;
  save_invstd[c] = invstd;
  const float sc = gamma ? gamma[c] * invstd : invstd;
  scale[c] = sc;
  shift[c] = (beta ? beta[c] : 0.f) - (float)mean * sc;
  if (running_mean) {
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
    const double unb = M > 1 ? var * M / (M - 1) : var;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unb;
  }
}

// per-channel parameter row r[c0 .. c0+V) (NULL: dflt) with 16-byte loads (c0 % 4 == 0 and
// the rows start 16-byte aligned)
template <int V>
__device__ __forceinline__ void ld_chan_row(const float* r, int c0, float dflt, float v[V]) {
  if (r) {
#pragma unroll
    for (int e = 0; e < V; e += 4) ld4(r + c0 + e, v + e);
  } else {
#pragma unroll
    for (int e = 0; e < V; ++e) v[e] = dflt;
  }
}

// The grid stride (gridDim*NT) is a multiple of tpp = C/V (a power of two <= NT),
// so each thread keeps one channel chunk: per-channel parameters live in registers.
// The f16 x3 pixel operand of the next conv, written by the f32 BN apply itself (dg_bn_apply_pair):
// the conv_fwd_psplit_kernel SCH 8 image [pixel][C / 32][hi 32 x f16 | lo 32 x f16] of y * 2^e, so the
// conv neither splits in-kernel nor runs split_x_h_kernel.  The scale must exist before y does, so e
// comes from a bound instead of max |y|: with the batch statistics over `count` pixels,
// |z - mean| <= sqrt(count) * sigma <= sqrt(count) / invstd, hence
//   |y_c| <= |scale_c| sqrt(count) / invstd_c + |shift_c + mean_c scale_c|   (= |gamma| sqrt(n) + |beta|),
// and ReLU only shrinks it.  2^e from the largest channel bound (h16_exp, as the conv's own scale from
// max |y|); the looser scale moves the parts' subnormal floor up by the bound's slack (2^7-2^10 here),
// far under the f32 rounding of the products.  Every block forms the same bound; block 0
// stores it for the conv (its xamax).
template <int NTB>
__device__ __forceinline__ float bn_pair_bound(const float* __restrict__ scale, const float* __restrict__ shift,
                                               const float* __restrict__ mean, const float* __restrict__ invstd,
                                               int C, double count) {
  __shared__ float red[NTB / 64];
  const float rn = (float)sqrt(count);
  float b = 0.f;
  for (int c = threadIdx.x; c < C; c += NTB)
    b = fmaxf(b, fabsf(scale[c]) * rn / invstd[c] + fabsf(fmaf(mean[c], scale[c], shift[c])));
  b = wave_max(b);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int w = 1; w < NTB / 64; ++w) r = fmaxf(r, red[w]);
  return r;
}
// 4 channels c0 .. c0 + 3 of one pixel row of the pair image
__device__ __forceinline__ void bn_pair_store(unsigned char* __restrict__ pair, long long p, int C, int c0,
                                              const float (&v)[4], float s) {
  unsigned h0, l0, h1, l1;
  split2h_pair(v[0], v[1], s, h0, l0);
  split2h_pair(v[2], v[3], s, h1, l1);
  unsigned char* d = pair + (p * (C >> 5) + (c0 >> 5)) * 128 + (c0 & 31) * 2;
  *(u2v*)d = u2v{h0, h1};
  *(u2v*)(d + 64) = u2v{l0, l1};
}

// PAIR (f32, 1024-thread form): also the f16 x3 pair image of y (bn_pair_bound above)
template <typename T, int U, int NTB = NT, int PAIR = 0>
__global__ __launch_bounds__(NTB) void bn_apply_kernel(const T* __restrict__ z, long long ldz, int M, int C,
                                                      const float* __restrict__ scale, const float* __restrict__ shift,
                                                      int act, const float* __restrict__ drop, int HW,
                                                      T* __restrict__ y, long long ldy, float* __restrict__ amax,
                                                      const float* __restrict__ mean = nullptr,
                                                      const float* __restrict__ invstd = nullptr, double count = 0.0,
                                                      unsigned char* __restrict__ pair = nullptr,
                                                      float* __restrict__ pbound = nullptr) {
  static_assert(!PAIR || (sizeof(T) == 4 && U == 1), "PAIR: the f32 BN apply");
  constexpr int V = 16 / (int)sizeof(T);
  const int tpp = C / V;
  const long long gt = blockIdx.x * (long long)NTB + threadIdx.x;
  const int c0 = (int)(gt % tpp) * V;
  const long long pstride = (long long)gridDim.x * NTB / tpp;
  float sc[V], sf[V];
  ld_chan_row<V>(scale, c0, 1.f, sc);
  ld_chan_row<V>(shift, c0, 0.f, sf);
  OutMax<T, V> m;  // max |y| per channel (amax: the f16 x3 convs' operand scales)
  float ps = 0.f;
  if constexpr (PAIR) {
    const float bnd = bn_pair_bound<NTB>(scale, shift, mean, invstd, C, count);
    ps = ldexpf(1.f, h16_exp(bnd));
    if (blockIdx.x == 0 && threadIdx.x == 0) *pbound = bnd;
  }
  auto apply = [&](long long p, float (&v)[V]) {
#pragma unroll
    for (int e = 0; e < V; ++e) {
      float t = fmaf(v[e], sc[e], sf[e]);
      if (act == 1) t = t > 0.f ? t : 0.f;
      v[e] = t;
    }
    if (drop) {
      const float* d = drop + (p / HW) * C + c0;
#pragma unroll
      for (int e = 0; e < V; ++e) v[e] *= d[e];
    }
    stv(y + p * ldy + c0, v);
    if constexpr (PAIR) bn_pair_store(pair, p, C, c0, v, ps);
#pragma unroll
    for (int e = 0; e < V; ++e) m.add(e, v[e]);
  };
  long long p = gt / tpp;
  // U pixels per trip, every load issued before the first use (DGVCC_EW_UNROLL)
  for (; p + (U - 1) * pstride < M; p += U * pstride) {
    float v[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) ldv(z + (p + u * pstride) * ldz + c0, v[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) apply(p + u * pstride, v[u]);
  }
  if constexpr (U > 1) {
    for (; p < M; p += pstride) {
      float v[V];
      ldv(z + p * ldz + c0, v);
      apply(p, v);
    }
  }
  if (amax) m.commit(c0, C, amax);
}

// Per-thread channel-chunk parameters (registers).
template <int V>
struct ChanParams {
  float sc[V], sf[V], mu[V], is[V];
  __device__ __forceinline__ void load(int c0, const float* scale, const float* shift, const float* mean,
                                       const float* invstd) {
    // NULL = identity (conv + activation without normalisation)
    ldrow(scale, c0, 1.f, sc);
    ldrow(shift, c0, 0.f, sf);
    ldrow(mean, c0, 0.f, mu);
    ldrow(invstd, c0, 1.f, is);
  }
  static __device__ __forceinline__ void ldrow(const float* r, int c0, float dflt, float v[V]) {
    ld_chan_row<V>(r, c0, dflt, v);
  }
};

// masked upstream gradient: g * drop, zeroed where the ReLU was inactive
// (relu mask recomputed from z exactly as the forward: fmaf(z, scale, shift) > 0)
template <int V>
__device__ __forceinline__ void bn_bwd_mask(long long p, int c0, int C, const ChanParams<V>& cp, int act,
                                            const float* drop, int HW, float gv[], const float zv[]) {
  if (drop) {
    const float* d = drop + (p / HW) * C + c0;
#pragma unroll
    for (int e = 0; e < V; ++e) gv[e] *= d[e];
  }
  if (act == 1) {
#pragma unroll
    for (int e = 0; e < V; ++e)
      if (!(fmaf(zv[e], cp.sc[e], cp.sf[e]) > 0.f)) gv[e] = 0.f;
  }
}
template <int V, bool DROP, bool ACT>
__device__ __forceinline__ void bn_mask_t(long long p, int c0, int C, const ChanParams<V>& cp, const float* drop,
                                          int HW, float gv[], const float zv[]) {
  if constexpr (DROP) {
    const float* d = drop + (p / HW) * C + c0;
#pragma unroll
    for (int e = 0; e < V; ++e) gv[e] *= d[e];
  }
  if constexpr (ACT) {
#pragma unroll
    for (int e = 0; e < V; ++e)
      if (!(fmaf(zv[e], cp.sc[e], cp.sf[e]) > 0.f)) gv[e] = 0.f;
  }
}
template <typename T, int V>
__device__ __forceinline__ void bn_bwd_load(const T* g, long long ldg, const T* z, long long ldz, long long p, int c0,
                                            int C, const ChanParams<V>& cp, int act, const float* drop, int HW,
                                            float gv[], float zv[]) {
  ldv(g + p * ldg + c0, gv);
  ldv(z + p * ldz + c0, zv);
  bn_bwd_mask<V>(p, c0, C, cp, act, drop, HW, gv, zv);
}

// DGVCC_EW_UNROLL=2: the channel-stationary elementwise passes handle two pixels per loop trip
// with all four loads issued before the first use; 1 (default): one pixel per trip
// (tools/bench_bn.py: two per trip is 2-7% slower at 94 VGPRs / 5 waves).  4 (BN apply only) and 2
// re-measured on the 1024-block grids in round 6 (profiles/round6d/bn_unroll.txt): still slower on
// every shape (f32 786432 x 256 BN apply 0.303 / 0.327 / 0.366 ms at 1 / 2 / 4)
inline int ew_unroll() {  // read per launch: same-process A/B (tools/bench_bn.py)
  const char* e = getenv("DGVCC_EW_UNROLL");
  return e && e[0] == '2' ? 2 : e && e[0] == '4' ? 4 : 1;
}

// gpart (f32, may be NULL): the block's max |g'| per channel, gpart[block][C] (dg_bn_bwd_pair's bound)
template <typename T>
__global__ __launch_bounds__(NT, sizeof(T) == 2 ? 7 : 1) void bn_bwd_partial(const T* __restrict__ g, long long ldg, const T* __restrict__ z,
                                                     long long ldz, int M, int C, int ppb, const float* mean,
                                                     const float* invstd, const float* scale, const float* shift,
                                                     int act, const float* drop, int HW, float* __restrict__ part,
                                                     float* __restrict__ gpart = nullptr) {
  constexpr int V = 16 / (int)sizeof(T);
  __shared__ float sh[3][NT * V];
  __shared__ float shm[sizeof(T) == 4 ? NT * V : 1];
  float gm[V];
#pragma unroll
  for (int e = 0; e < V; ++e) gm[e] = 0.f;
  const int tpp = C / V;
  const int rows = NT / tpp;
  const int tid = threadIdx.x;
  const int ch = tid % tpp, pl = tid / tpp;
  const int c0 = ch * V;
  float sg[V], sgx[V], sx[V];
#pragma unroll
  for (int e = 0; e < V; ++e) { sg[e] = 0.f; sgx[e] = 0.f; sx[e] = 0.f; }
  const int p0 = blockIdx.x * ppb, p1 = min(M, p0 + ppb);
  if (pl < rows) {
    ChanParams<V> cp;
    cp.load(c0, scale, shift, mean, invstd);
    if constexpr (V == 8) {
      // 16-bit: sum g' z and z in the loop and centre once per thread afterwards
      // (sum g' xhat = (sum g' z - mu sum g') is, sum xhat = (sum z - n mu) is), so mean / invstd
      // are not held across the loop (92 -> <= 72 VGPRs: 7 waves per SIMD instead of 5); the
      // per-thread sums run over a few hundred pixels, far inside f32 for 16-bit operands
      int cnt = 0;
      for (int p = p0 + pl; p < p1; p += rows) {
        float gv[V], zv[V];
        bn_bwd_load<T, V>(g, ldg, z, ldz, p, c0, C, cp, act, drop, HW, gv, zv);
#pragma unroll
        for (int e = 0; e < V; ++e) {
          sg[e] += gv[e];
          sgx[e] = fmaf(gv[e], zv[e], sgx[e]);
          sx[e] += zv[e];
        }
        ++cnt;
      }
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float mu = mean ? mean[c0 + e] : 0.f, is = invstd ? invstd[c0 + e] : 1.f;
        sgx[e] = (sgx[e] - mu * sg[e]) * is;
        sx[e] = (sx[e] - (float)cnt * mu) * is;
      }
    } else {
      for (int p = p0 + pl; p < p1; p += rows) {
        float gv[V], zv[V];
        bn_bwd_load<T, V>(g, ldg, z, ldz, p, c0, C, cp, act, drop, HW, gv, zv);
#pragma unroll
        for (int e = 0; e < V; ++e) {
          const float xh = (zv[e] - cp.mu[e]) * cp.is[e];
          sg[e] += gv[e];
          sgx[e] = fmaf(gv[e], xh, sgx[e]);
          sx[e] += xh;
          gm[e] = fmaxf(gm[e], fabsf(gv[e]));
        }
      }
    }
#pragma unroll
    for (int e = 0; e < V; ++e) {
      sh[0][pl * C + c0 + e] = sg[e];
      sh[1][pl * C + c0 + e] = sgx[e];
      sh[2][pl * C + c0 + e] = sx[e];
      if constexpr (sizeof(T) == 4) shm[pl * C + c0 + e] = gm[e];
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += NT) {
    float a = 0.f, b = 0.f, d = 0.f;
    for (int r = 0; r < rows; ++r) { a += sh[0][r * C + c]; b += sh[1][r * C + c]; d += sh[2][r * C + c]; }
    float* o = part + (long long)blockIdx.x * 3 * C;
    o[c] = a; o[C + c] = b; o[2 * C + c] = d;
    if constexpr (sizeof(T) == 4) {
      if (gpart) {
        float mx = 0.f;
        for (int r = 0; r < rows; ++r) mx = fmaxf(mx, shm[r * C + c]);
        gpart[(long long)blockIdx.x * C + c] = mx;
      }
    }
  }
}

// gpart / bpart (may be NULL): the per-block max |g'| rows of bn_bwd_partial -> bpart[blockIdx.x] = the
// largest over this block's 16 channels of |k1| max |g'| + |k2| sqrt(count) + |k3| >= max |dz| (|xhat| <=
// sqrt(count) for batch statistics over count pixels): dg_bn_bwd_pair's pair-image scale bound
__global__ __launch_bounds__(NT) void bn_bwd_finalize(const float* __restrict__ part, int nblk, int M, int C,
                                                      const float* gamma, const float* invstd, float* dgamma,
                                                      float* dbeta, float* dbias, float* coef,
                                                      const float* __restrict__ gpart = nullptr,
                                                      float* __restrict__ bpart = nullptr, double count = 0.0) {
  __shared__ double sh[3][16][17];
  __shared__ float shg[16][17];
  const int cl = threadIdx.x & 15, r = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  double a = 0.0, b = 0.0, d = 0.0;
  float gmx = 0.f;
  if (gpart && c < C) {
    int k = r;
    for (; k + 48 < nblk; k += 64) {  // four rows in flight (as the sums below)
      float v4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v4[u] = gpart[(long long)(k + 16 * u) * C + c];
#pragma unroll
      for (int u = 0; u < 4; ++u) gmx = fmaxf(gmx, v4[u]);
    }
    for (; k < nblk; k += 16) gmx = fmaxf(gmx, gpart[(long long)k * C + c]);
  }
  shg[r][cl] = gmx;
  if (c < C) {
    int k = r;
    for (; k + 48 < nblk; k += 64) {
      float a4[4], b4[4], d4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* o = part + (long long)(k + 16 * u) * 3 * C;
        a4[u] = o[c]; b4[u] = o[C + c]; d4[u] = o[2 * C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { a += a4[u]; b += b4[u]; d += d4[u]; }
    }
    for (; k < nblk; k += 16) {
      const float* o = part + (long long)k * 3 * C;
      a += o[c]; b += o[C + c]; d += o[2 * C + c];
    }
  }
  sh[0][r][cl] = a; sh[1][r][cl] = b; sh[2][r][cl] = d;
  __syncthreads();
  if (r != 0) return;
  float bnd = 0.f;  // this channel's |dz| bound (bpart)
  if (c < C) {
    a = 0.0; b = 0.0; d = 0.0;
    for (int q = 0; q < 16; ++q) { a += sh[0][q][cl]; b += sh[1][q][cl]; d += sh[2][q][cl]; }
    float gmax = 0.f;
    for (int q = 0; q < 16; ++q) gmax = fmaxf(gmax, shg[q][cl]);
    if (!invstd) {  // no normalisation: dz = act'(z) g ; dbeta = dbias = sum dz
      if (dgamma) dgamma[c] = 0.f;
      if (dbeta) dbeta[c] = (float)a;
      if (dbias) dbias[c] = (float)a;
      coef[c] = 1.f; coef[C + c] = 0.f; coef[2 * C + c] = 0.f;
      bnd = gmax;
    } else {
      const float gm = gamma ? gamma[c] : 1.f;
      const float k1 = gm * invstd[c];
      const float k2 = (float)(k1 * b / M);
      const float k3 = (float)(k1 * a / M);
      if (dgamma) dgamma[c] = (float)b;
      if (dbeta) dbeta[c] = (float)a;
      if (dbias) dbias[c] = (float)(-(double)k2 * d);
      coef[c] = k1; coef[C + c] = k2; coef[2 * C + c] = k3;
      bnd = fabsf(k1) * gmax + fabsf(k2) * (float)sqrt(count) + fabsf(k3);
    }
  }
  if (bpart) {  // lanes 0-15 of wave 0: the block's largest
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) bnd = fmaxf(bnd, __shfl_xor(bnd, o, 16));
    if (cl == 0) bpart[blockIdx.x] = bnd;
  }
}

// Column sums of part[nblk][3][C] in double -> out[3][C] (a rank's BN-backward sums, fixed order).
__global__ __launch_bounds__(NT) void bn_sum_rows3(const float* __restrict__ part, int nblk, int C,
                                                   float* __restrict__ out) {
  __shared__ double sh[3][16][17];
  const int cl = threadIdx.x & 15, r = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  double a = 0.0, b = 0.0, d = 0.0;
  if (c < C)
    for (int k = r; k < nblk; k += 16) {
      const float* o = part + (long long)k * 3 * C;
      a += o[c]; b += o[C + c]; d += o[2 * C + c];
    }
  sh[0][r][cl] = a; sh[1][r][cl] = b; sh[2][r][cl] = d;
  __syncthreads();
  if (r != 0 || c >= C) return;
  a = 0.0; b = 0.0; d = 0.0;
  for (int q = 0; q < 16; ++q) { a += sh[0][q][cl]; b += sh[1][q][cl]; d += sh[2][q][cl]; }
  out[c] = (float)a; out[C + c] = (float)b; out[2 * C + c] = (float)d;
}

// SyncBatchNorm backward finalize (torch.nn.SyncBatchNorm semantics): the dz coefficients from the
// sums over all ranks (sg = sum g', sgx = sum g' xhat over Mg pixels), dgamma / dbeta from this
// rank's sums (data parallel then averages them with the other parameter gradients), and the conv
// bias gradient as this rank's sum of dz: k1 sg_l - k2 sx_l - Ml k3.
__global__ __launch_bounds__(NT) void bn_bwd_finalize_sync(const float* __restrict__ loc, const float* __restrict__ glob,
                                                           int Ml, double Mg, int C, const float* gamma,
                                                           const float* invstd, float* dgamma, float* dbeta,
                                                           float* dbias, float* coef) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= C) return;
  // Mg <= 0: the pixel count over all ranks is the all-reduced fourth row (hi + lo parts, each
  // exact in f32), so ranks holding different batch sizes share one count, as in the forward
  if (Mg <= 0.0) Mg = (double)glob[3 * C] + (double)glob[3 * C + 1];
  const float gm = gamma ? gamma[c] : 1.f;
  const float k1 = gm * invstd[c];
  const float k2 = (float)(k1 * (double)glob[C + c] / Mg);
  const float k3 = (float)(k1 * (double)glob[c] / Mg);
  if (dgamma) dgamma[c] = loc[C + c];
  if (dbeta) dbeta[c] = loc[c];
  if (dbias) dbias[c] = (float)((double)k1 * loc[c] - (double)k2 * loc[2 * C + c] - (double)Ml * k3);
  coef[c] = k1; coef[C + c] = k2; coef[2 * C + c] = k3;
}

// The max over nb bound partials (bn_bwd_finalize bpart), every block alike
template <int NTB>
__device__ __forceinline__ float bn_bpart_max(const float* __restrict__ bpart, int nb) {
  __shared__ float red[NTB / 64];
  float b = 0.f;
  for (int i = threadIdx.x; i < nb; i += NTB) b = fmaxf(b, bpart[i]);
  b = wave_max(b);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int w = 1; w < NTB / 64; ++w) r = fmaxf(r, red[w]);
  return r;
}

// PAIR (f32, 1024-thread form): also the f16 x3 pair image of dz for the dgrad (dg_bn_bwd_pair), its
// scale from the bound partials (bn_bwd_finalize bpart)
template <typename T, int U = 1, int NTB = NT, int PAIR = 0>
__global__ __launch_bounds__(NTB, NTB == NT && sizeof(T) == 2 ? (U == 2 ? 1 : 7) : 1) void bn_bwd_apply(const T* __restrict__ g, long long ldg, const T* __restrict__ z,
                                                   long long ldz, int M, int C, const float* mean, const float* invstd,
                                                   const float* scale, const float* shift, int act, const float* drop,
                                                   int HW, const float* __restrict__ coef, T* __restrict__ dz,
                                                   long long lddz, float* __restrict__ amax,
                                                   const float* __restrict__ bpart = nullptr, int nbp = 0,
                                                   unsigned char* __restrict__ pair = nullptr,
                                                   float* __restrict__ pbound = nullptr) {
  static_assert(!PAIR || (sizeof(T) == 4 && U == 1), "PAIR: the f32 BN backward apply");
  constexpr int V = 16 / (int)sizeof(T);
  OutMax<T, V> m;  // max |dz| per channel (amax)
  const int tpp = C / V;
  const long long gt = blockIdx.x * (long long)NTB + threadIdx.x;
  const int c0 = (int)(gt % tpp) * V;
  const long long pstride = (long long)gridDim.x * NTB / tpp;
  ChanParams<V> cp;
  cp.load(c0, scale, shift, mean, invstd);
  float k1[V], k2[V], k3[V];
  ChanParams<V>::ldrow(coef, c0, 0.f, k1);
  ChanParams<V>::ldrow(coef + C, c0, 0.f, k2);
  ChanParams<V>::ldrow(coef + 2 * C, c0, 0.f, k3);
  if constexpr (V == 8) {
    // 16-bit: dz = k1 g' - (k2 is) z + (k2 is mu - k3), with k1 = gamma * invstd = the forward's
    // scale (every finalizer forms both as that one product; identity when unnormalised), so 4
    // per-channel values stay in registers instead of 7 (90 -> 64 VGPRs: 8 waves per SIMD
    // instead of 5).  The result is rounded to 16 bits; the f32 reassociation is far below that.
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const float A = k2[e] * cp.is[e];
      k3[e] = A * cp.mu[e] - k3[e];
      k2[e] = A;
    }
  }
  auto f = [&](float gv[], const float zv[]) {
#pragma unroll
    for (int e = 0; e < V; ++e) {
      if constexpr (V == 8) {
        gv[e] = fmaf(cp.sc[e], gv[e], fmaf(-k2[e], zv[e], k3[e]));
      } else {
        const float xh = (zv[e] - cp.mu[e]) * cp.is[e];
        gv[e] = k1[e] * gv[e] - k2[e] * xh - k3[e];
      }
    }
  };
  // dropout / ReLU as compile-time flags: straight-line loop bodies (no loads behind branches)
  auto run = [&](auto drop_t, auto act_t) {
    constexpr bool DROP = decltype(drop_t)::value, ACT = decltype(act_t)::value;
    long long p = gt / tpp;
    if constexpr (U == 2) {
      for (; p + pstride < M; p += 2 * pstride) {
        const long long q = p + pstride;
        float g0[V], z0[V], g1[V], z1[V];
        ldv(g + p * ldg + c0, g0);
        ldv(z + p * ldz + c0, z0);
        ldv(g + q * ldg + c0, g1);
        ldv(z + q * ldz + c0, z1);
        bn_mask_t<V, DROP, ACT>(p, c0, C, cp, drop, HW, g0, z0);
        bn_mask_t<V, DROP, ACT>(q, c0, C, cp, drop, HW, g1, z1);
        f(g0, z0);
        f(g1, z1);
        stv(dz + p * lddz + c0, g0);
        stv(dz + q * lddz + c0, g1);
#pragma unroll
        for (int e = 0; e < V; ++e) { m.add(e, g0[e]); m.add(e, g1[e]); }
      }
    }
    for (; p < M; p += pstride) {
      float gv[V], zv[V];
      ldv(g + p * ldg + c0, gv);
      ldv(z + p * ldz + c0, zv);
      bn_mask_t<V, DROP, ACT>(p, c0, C, cp, drop, HW, gv, zv);
      f(gv, zv);
      stv(dz + p * lddz + c0, gv);
#pragma unroll
      for (int e = 0; e < V; ++e) m.add(e, gv[e]);
    }
  };
  if constexpr (U == 1) {  // the round-3 loop (runtime dropout / ReLU flags)
    float ps = 0.f;
    if constexpr (PAIR) {
      const float bnd = bn_bpart_max<NTB>(bpart, nbp);
      ps = ldexpf(1.f, h16_exp(bnd));
      if (blockIdx.x == 0 && threadIdx.x == 0) *pbound = bnd;
    }
    for (long long p = gt / tpp; p < M; p += pstride) {
      float gv[V], zv[V];
      bn_bwd_load<T, V>(g, ldg, z, ldz, p, c0, C, cp, act, drop, HW, gv, zv);
      f(gv, zv);
      stv(dz + p * lddz + c0, gv);
      if constexpr (PAIR) bn_pair_store(pair, p, C, c0, gv, ps);
#pragma unroll
      for (int e = 0; e < V; ++e) m.add(e, gv[e]);
    }
  } else if (drop) {
    if (act == 1) run(std::true_type{}, std::true_type{});
    else run(std::true_type{}, std::false_type{});
  } else {
    if (act == 1) run(std::false_type{}, std::true_type{});
    else run(std::false_type{}, std::false_type{});
  }
  if (amax) m.commit(c0, C, amax);
}

// ---------------------------------------------------------------------------
// BN(+ReLU) fused with the following MaxPool2d(2, 2) (vgg16_bn.features[5:7],
// [12:14], [22:24], [32:34]; models/models.py:35-38).  One thread = one pooled
// pixel x one 16-B channel chunk; the 2x2 window's four z vectors give the four
// activations y_k = rnd(act(z*scale + shift) * drop) exactly as bn_apply_kernel
// stores them, and the pooled value is their first-max (ATen scan order, NaN
// propagates).  The backward recomputes the same y_k to route the pooled
// gradient to the window's argmax, so neither y nor the full-resolution
// gradient of y is ever materialised (only a direct full-resolution gradient,
// when y also feeds another consumer, e.g. x1/x2 into the decoder concats).
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ float rnd_t(float v) { return to_f(from_f<T>(v)); }

__device__ __forceinline__ void pool_window(long long pp, int H, int W, long long pos[4]) {
  const int Ho = H / 2, Wo = W / 2;
  const int p32 = (int)pp;  // N*H*W < 2^31 (checked by the ABI): 32-bit division
  const int wo = p32 % Wo;
  const int t = p32 / Wo;
  const int ho = t % Ho;
  const int n = t / Ho;
  const long long p00 = ((long long)n * H + 2 * ho) * W + 2 * wo;
  pos[0] = p00; pos[1] = p00 + 1; pos[2] = p00 + W; pos[3] = p00 + W + 1;
}

// first max of the four window values (same rule as resample.hip argmax4)
__device__ __forceinline__ int first_max4(float a, float b, float c, float d) {
  int k = 0;
  float m = a;
  if (b > m || isnan(b)) { m = b; k = 1; }
  if (c > m || isnan(c)) { m = c; k = 2; }
  if (d > m || isnan(d)) { m = d; k = 3; }
  return k;
}

// PAIR (f32, 1024-thread form): also the f16 x3 pair image of the pooled yp (the bound of y bounds it)
template <typename T, int NTB = NT, int PAIR = 0>
__global__ __launch_bounds__(NTB) void bn_apply_pool_kernel(const T* __restrict__ z, long long ldz, int H, int W,
                                                           long long Mp, int C, const float* __restrict__ scale,
                                                           const float* __restrict__ shift, int act,
                                                           const float* __restrict__ drop, int HW, T* __restrict__ y,
                                                           long long ldy, T* __restrict__ yp, long long ldyp,
                                                           float* __restrict__ amax,
                                                           const float* __restrict__ mean = nullptr,
                                                           const float* __restrict__ invstd = nullptr,
                                                           double count = 0.0, unsigned char* __restrict__ pair = nullptr,
                                                           float* __restrict__ pbound = nullptr) {
  static_assert(!PAIR || sizeof(T) == 4, "PAIR: the f32 pooled BN apply");
  constexpr int V = 16 / (int)sizeof(T);
  OutMax<T, V> m;  // max |y| per channel over the window values (>= max |yp|: amax of both)
  const int tpp = C / V;
  const long long gt = blockIdx.x * (long long)NTB + threadIdx.x;
  const int c0 = (int)(gt % tpp) * V;
  const long long pstride = (long long)gridDim.x * NTB / tpp;
  float sc[V], sf[V];
  ld_chan_row<V>(scale, c0, 1.f, sc);
  ld_chan_row<V>(shift, c0, 0.f, sf);
  float ps = 0.f;
  if constexpr (PAIR) {
    const float bnd = bn_pair_bound<NTB>(scale, shift, mean, invstd, C, count);
    ps = ldexpf(1.f, h16_exp(bnd));
    if (blockIdx.x == 0 && threadIdx.x == 0) *pbound = bnd;
  }
  for (long long pp = gt / tpp; pp < Mp; pp += pstride) {
    long long pos[4];
    pool_window(pp, H, W, pos);
    float v[4][V];
#pragma unroll
    for (int k = 0; k < 4; ++k) ldv(z + pos[k] * ldz + c0, v[k]);
    const float* d = drop ? drop + (pos[0] / HW) * C + c0 : nullptr;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        float t = fmaf(v[k][e], sc[e], sf[e]);
        if (act == 1) t = t > 0.f ? t : 0.f;
        if (d) t *= d[e];
        v[k][e] = rnd_t<T>(t);
        m.add(e, v[k][e]);
      }
      if (y) stv(y + pos[k] * ldy + c0, v[k]);
    }
    float o[V];
#pragma unroll
    for (int e = 0; e < V; ++e) o[e] = v[first_max4(v[0][e], v[1][e], v[2][e], v[3][e])][e];
    stv(yp + pp * ldyp + c0, o);
    if constexpr (PAIR) bn_pair_store(pair, pp, C, c0, o, ps);
  }
  if (amax) m.commit(c0, C, amax);
}

// The pooled backward keeps 4 pixels x V channels of z and g live per thread: V = 4
// (8-B bf16 loads) holds the two kernels under ~100 VGPRs, 4-5 waves per SIMD instead of 2
// at V = 8, which is what a latency-bound gather of 4 rows needs.
constexpr int POOL_V = 4;
template <int V, typename T>
__device__ __forceinline__ void ldn(const T* p, float* v) {
  if constexpr (V == 4) ld4(p, v);
  else ldv(p, v);
}
template <int V, typename T>
__device__ __forceinline__ void stn(T* p, const float* v) {
  if constexpr (V == 4) st4(p, v);
  else stv(p, v);
}

// Upstream gradient of the BN output at the window's four pixels: the pooled
// gradient at the recomputed argmax (+ the direct gradient gd), times drop,
// zeroed where the ReLU was inactive (bn_bwd_load's rule).
template <typename T, int V>
__device__ __forceinline__ void bn_pool_bwd_load(const T* gp, long long ldgp, const T* gd, long long ldgd, const T* z,
                                                 long long ldz, long long pp, const long long pos[4], int c0, int C,
                                                 const ChanParams<V>& cp, int act, const float* drop, int HW,
                                                 float gv[4][V], float zv[4][V]) {
  float gpv[V];
  ldn<V>(gp + pp * ldgp + c0, gpv);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    ldn<V>(z + pos[k] * ldz + c0, zv[k]);
    if (gd) ldn<V>(gd + pos[k] * ldgd + c0, gv[k]);
    else {
#pragma unroll
      for (int e = 0; e < V; ++e) gv[k][e] = 0.f;
    }
  }
  const float* d = drop ? drop + (pos[0] / HW) * C + c0 : nullptr;
#pragma unroll
  for (int e = 0; e < V; ++e) {
    float y[4];
    bool on[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float t = fmaf(zv[k][e], cp.sc[e], cp.sf[e]);
      on[k] = t > 0.f;  // the ReLU mask of bn_bwd_load: fmaf(z, scale, shift) > 0
      if (act == 1) t = on[k] ? t : 0.f;
      if (d) t *= d[e];
      y[k] = rnd_t<T>(t);
    }
    const int am = first_max4(y[0], y[1], y[2], y[3]);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k == am) gv[k][e] += gpv[e];
      if (d) gv[k][e] *= d[e];
      if (act == 1 && !on[k]) gv[k][e] = 0.f;
    }
  }
}

// gpart (f32, may be NULL): as bn_bwd_partial
template <typename T>
__global__ __launch_bounds__(NT) void bn_pool_bwd_partial(const T* __restrict__ gp, long long ldgp,
                                                          const T* __restrict__ gd, long long ldgd,
                                                          const T* __restrict__ z, long long ldz, int H, int W,
                                                          long long Mp, int C, long long ppb, const float* mean,
                                                          const float* invstd, const float* scale, const float* shift,
                                                          int act, const float* drop, int HW, float* __restrict__ part,
                                                          float* __restrict__ gpart = nullptr) {
  constexpr int V = POOL_V;
  __shared__ float sh[3][NT * V];
  __shared__ float shm[sizeof(T) == 4 ? NT * V : 1];
  float gm[V];
#pragma unroll
  for (int e = 0; e < V; ++e) gm[e] = 0.f;
  const int tpp = C / V;
  const int rows = NT / tpp;
  const int tid = threadIdx.x;
  const int ch = tid % tpp, pl = tid / tpp;
  const int c0 = ch * V;
  float sg[V], sgx[V], sx[V];
#pragma unroll
  for (int e = 0; e < V; ++e) { sg[e] = 0.f; sgx[e] = 0.f; sx[e] = 0.f; }
  const long long p0 = blockIdx.x * ppb, p1 = min(Mp, p0 + ppb);
  if (pl < rows) {
    ChanParams<V> cp;
    cp.load(c0, scale, shift, mean, invstd);
    for (long long pp = p0 + pl; pp < p1; pp += rows) {
      long long pos[4];
      pool_window(pp, H, W, pos);
      float gv[4][V], zv[4][V];
      bn_pool_bwd_load<T, V>(gp, ldgp, gd, ldgd, z, ldz, pp, pos, c0, C, cp, act, drop, HW, gv, zv);
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < V; ++e) {
          const float xh = (zv[k][e] - cp.mu[e]) * cp.is[e];
          sg[e] += gv[k][e];
          sgx[e] = fmaf(gv[k][e], xh, sgx[e]);
          sx[e] += xh;
          if constexpr (sizeof(T) == 4) gm[e] = fmaxf(gm[e], fabsf(gv[k][e]));
        }
    }
#pragma unroll
    for (int e = 0; e < V; ++e) {
      sh[0][pl * C + c0 + e] = sg[e];
      sh[1][pl * C + c0 + e] = sgx[e];
      sh[2][pl * C + c0 + e] = sx[e];
      if constexpr (sizeof(T) == 4) shm[pl * C + c0 + e] = gm[e];
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += NT) {
    float a = 0.f, b = 0.f, d = 0.f;
    for (int r = 0; r < rows; ++r) { a += sh[0][r * C + c]; b += sh[1][r * C + c]; d += sh[2][r * C + c]; }
    float* o = part + (long long)blockIdx.x * 3 * C;
    o[c] = a; o[C + c] = b; o[2 * C + c] = d;
    if constexpr (sizeof(T) == 4) {
      if (gpart) {
        float mx = 0.f;
        for (int r = 0; r < rows; ++r) mx = fmaxf(mx, shm[r * C + c]);
        gpart[(long long)blockIdx.x * C + c] = mx;
      }
    }
  }
}

// PAIR (f32, 1024-thread form): also the pair image of dz (as bn_bwd_apply)
template <typename T, int NTB = NT, int PAIR = 0>
__global__ __launch_bounds__(NTB) void bn_pool_bwd_apply(const T* __restrict__ gp, long long ldgp,
                                                        const T* __restrict__ gd, long long ldgd,
                                                        const T* __restrict__ z, long long ldz, int H, int W,
                                                        long long Mp, int C, const float* mean, const float* invstd,
                                                        const float* scale, const float* shift, int act,
                                                        const float* drop, int HW, const float* __restrict__ coef,
                                                        T* __restrict__ dz, long long lddz, float* __restrict__ amax,
                                                        const float* __restrict__ bpart = nullptr, int nbp = 0,
                                                        unsigned char* __restrict__ pair = nullptr,
                                                        float* __restrict__ pbound = nullptr) {
  static_assert(!PAIR || sizeof(T) == 4, "PAIR: the f32 pooled BN backward apply");
  constexpr int V = POOL_V;
  OutMax<T, V> m;  // max |dz| per channel
  const int tpp = C / V;
  const long long gt = blockIdx.x * (long long)NTB + threadIdx.x;
  const int c0 = (int)(gt % tpp) * V;
  const long long pstride = (long long)gridDim.x * NTB / tpp;
  ChanParams<V> cp;
  cp.load(c0, scale, shift, mean, invstd);
  float k1[V], k2[V], k3[V];
  ld_chan_row<V>(coef, c0, 0.f, k1);
  ld_chan_row<V>(coef + C, c0, 0.f, k2);
  ld_chan_row<V>(coef + 2 * C, c0, 0.f, k3);
  float ps = 0.f;
  if constexpr (PAIR) {
    const float bnd = bn_bpart_max<NTB>(bpart, nbp);
    ps = ldexpf(1.f, h16_exp(bnd));
    if (blockIdx.x == 0 && threadIdx.x == 0) *pbound = bnd;
  }
  for (long long pp = gt / tpp; pp < Mp; pp += pstride) {
    long long pos[4];
    pool_window(pp, H, W, pos);
    float gv[4][V], zv[4][V];
    bn_pool_bwd_load<T, V>(gp, ldgp, gd, ldgd, z, ldz, pp, pos, c0, C, cp, act, drop, HW, gv, zv);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float xh = (zv[k][e] - cp.mu[e]) * cp.is[e];
        gv[k][e] = k1[e] * gv[k][e] - k2[e] * xh - k3[e];
        m.add(e, gv[k][e]);
      }
      stn<V>(dz + pos[k] * lddz + c0, gv[k]);
      if constexpr (PAIR) bn_pair_store(pair, pos[k], C, c0, gv[k], ps);
    }
  }
  if (amax) m.commit(c0, C, amax);
}

inline int ew_grid(long long n) {
  long long g = (n + NT - 1) / NT;
  return (int)std::max<long long>(1, std::min<long long>(g, 8192));
}
// Grid of the channel-stationary passes (bn_apply_kernel, bn_bwd_apply): each thread loads its
// channel chunk's parameters once, so fewer, longer-lived threads amortise that prologue.
// DGVCC_EW_GRID (read per launch: tools/bench_bn.py) caps the blocks.
inline int cs_grid(long long n) {
  // tools/bench_bn.py: round 4 (profiles/round4a/bn_grid) took 16384 blocks where that left every
  // thread >= 2 chunks, else 2048; round 5 (profiles/round5b/bn_grid.txt), with the f32 passes
  // also folding max |out| for the f16 x3 convs: 1024 blocks (4 per CU) matched or beat both on
  // the trunk / encoder shapes in f32 and bf16 (bf16 12.6M x 64 BN backward 1.04 -> 0.93 ms,
  // f32 3.1M x 128 0.99 -> 0.89 ms)
  const char* e = getenv("DGVCC_EW_GRID");
  const long long g = (n + NT - 1) / NT;
  if (e) return (int)std::max<long long>(1, std::min<long long>(g, std::max(64, atoi(e))));
  return (int)std::min<long long>(g, 1024);
}

constexpr int EW_WIDE = DG_EW_WIDE;
inline bool ew_wide(const float* amax, bool f32) { return dg_ew_wide(amax, f32); }
inline int wide_grid(long long n, int cap) {
  return (int)std::max<long long>(1, std::min<long long>((n + EW_WIDE - 1) / EW_WIDE, cap));
}

template <typename T>
int bn_fwd_impl(const void* z, long long ldz, int M, int C, const float* gamma, const float* beta, float* rm, float* rv,
                float momentum, float eps, float* smean, float* sinv, float* scale, float* shift, void* ws,
                hipStream_t st) {
  const int nblk = bn_nblk(M);
  const int ppb = dg_cdiv(M, nblk);
  hipLaunchKernelGGL(bn_stats_partial<T>, dim3(nblk), dim3(NT), 0, st, (const T*)z, ldz, M, C, ppb, (float*)ws);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_stats_finalize<T>, dim3(dg_cdiv(C, 16)), dim3(NT), 0, st, (const T*)z, (const float*)ws,
                     nblk, M, C, gamma, beta, rm, rv, momentum, eps, smean, sinv, scale, shift);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// amax (may be NULL): max |out| of the apply pass, per channel for f32 (dg_common.h OutMax)
static int zero_amax(float* amax, bool f32, int C, hipStream_t st) {
  return dg_zero_amax(amax, f32 ? DG_F32 : DG_BF16, C, st);
}
template <typename T>
int bn_bwd_impl(const void* g, long long ldg, const void* z, long long ldz, int M, int C, const float* gamma,
                const float* mean, const float* inv, const float* scale, const float* shift, int act,
                const float* drop, int HW, void* dz, long long lddz, float* dgamma, float* dbeta, float* dbias,
                void* ws, hipStream_t st, float* coef_out = nullptr, float* amax = nullptr) {
  const int nblk = bn_nblk(M);
  const int ppb = dg_cdiv(M, nblk);
  float* part = (float*)ws;
  float* coef = coef_out ? coef_out : part + (long long)nblk * 3 * C;
  hipLaunchKernelGGL(bn_bwd_partial<T>, dim3(nblk), dim3(NT), 0, st, (const T*)g, ldg, (const T*)z, ldz, M, C, ppb,
                     mean, inv, scale, shift, act, drop, HW, part);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_bwd_finalize, dim3(dg_cdiv(C, 16)), dim3(NT), 0, st, part, nblk, M, C, gamma, inv, dgamma,
                     dbeta, dbias, coef);
  DG_CHECK_LAUNCH();
  if (!dz) return DG_OK;  // coefficients only (a fused consumer applies them)
  { const int zr = zero_amax(amax, sizeof(T) == 4, C, st); if (zr != DG_OK) return zr; }
  const long long total = (long long)M * (C / (16 / (int)sizeof(T)));
  if (ew_wide(amax, sizeof(T) == 4))
    hipLaunchKernelGGL((bn_bwd_apply<T, 1, EW_WIDE>), dim3(wide_grid(total, 256)), dim3(EW_WIDE), 0, st, (const T*)g, ldg,
                       (const T*)z, ldz, M, C, mean, inv, scale, shift, act, drop, HW, coef, (T*)dz, lddz, amax);
  else
    hipLaunchKernelGGL((ew_unroll() == 2 ? bn_bwd_apply<T, 2> : bn_bwd_apply<T, 1>), dim3(cs_grid(total)), dim3(NT), 0, st, (const T*)g, ldg, (const T*)z, ldz, M, C,
                       mean, inv, scale, shift, act, drop, HW, coef, (T*)dz, lddz, amax, nullptr, 0, nullptr, nullptr);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

}  // namespace

extern "C" int64_t dg_bn_workspace(int M, int C) {
  if (M <= 0 || C <= 0) return DG_ERR_INVALID;
  // partials [nblk][3][C], coef [3][C], and for the pair entries the max |g'| rows [nblk][C] and the
  // bound partials [C / 16]
  return ((int64_t)std::max(bn_nblk(M), pool_nblk(M / 4)) * 4 + 4) * C * 4 + 1024;
}

// C/V must divide NT (power of two <= 256): every thread then owns one channel chunk.
#define BN_SHAPE_OK(dtype, C, ld)                                                        \
  ((C) % (DG_IS16(dtype) ? 8 : 4) == 0 && NT % ((C) / (DG_IS16(dtype) ? 8 : 4)) == 0 && \
   (ld) % (DG_IS16(dtype) ? 8 : 4) == 0)

extern "C" int dg_bn_fwd_train(int dtype, const void* z, int64_t ldz, int M, int C, const float* gamma,
                               const float* beta, float* running_mean, float* running_var, float momentum, float eps,
                               float* save_mean, float* save_invstd, float* scale, float* shift, void* workspace,
                               void* stream) {
  DG_REQUIRE(z && save_mean && save_invstd && scale && shift && workspace && M > 0 && C > 0 && ldz >= C);
  DG_REQUIRE((running_mean == nullptr) == (running_var == nullptr));
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(BN_SHAPE_OK(dtype, C, ldz));
  hipStream_t st = (hipStream_t)stream;
  return dtype == DG_BF16 ? bn_fwd_impl<bf16>(z, ldz, M, C, gamma, beta, running_mean, running_var, momentum, eps,
                                              save_mean, save_invstd, scale, shift, workspace, st)
                          : dtype == DG_F16 ? bn_fwd_impl<f16>(z, ldz, M, C, gamma, beta, running_mean, running_var, momentum, eps,
                                              save_mean, save_invstd, scale, shift, workspace, st) : bn_fwd_impl<float>(z, ldz, M, C, gamma, beta, running_mean, running_var, momentum, eps,
                                               save_mean, save_invstd, scale, shift, workspace, st);
}

extern "C" int dg_bn_apply(int dtype, const void* z, int64_t ldz, int M, int C, const float* scale, const float* shift,
                           int act, const float* drop, int HW, void* y, int64_t ldy, float* amax, void* stream) {
  DG_REQUIRE(z && y && scale && shift && M > 0 && C > 0 && ldz >= C && ldy >= C && (act == 0 || act == 1));
  DG_REQUIRE(!drop || HW > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(BN_SHAPE_OK(dtype, C, ldz) && BN_SHAPE_OK(dtype, C, ldy));
  hipStream_t st = (hipStream_t)stream;
  { const int zr = zero_amax(amax, dtype == DG_F32, C, st); if (zr != DG_OK) return zr; }
  const long long total = (long long)M * (C / (DG_IS16(dtype) ? 8 : 4));
  if (dtype == DG_BF16)
    hipLaunchKernelGGL((ew_unroll() == 4 ? bn_apply_kernel<bf16, 4> : ew_unroll() == 2 ? bn_apply_kernel<bf16, 2> : bn_apply_kernel<bf16, 1>), dim3(cs_grid(total)), dim3(NT), 0, st, (const bf16*)z, ldz, M, C, scale,
                       shift, act, drop, HW, (bf16*)y, ldy, amax, nullptr, nullptr, 0.0, nullptr, nullptr);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL((ew_unroll() == 4 ? bn_apply_kernel<f16, 4> : ew_unroll() == 2 ? bn_apply_kernel<f16, 2> : bn_apply_kernel<f16, 1>), dim3(cs_grid(total)), dim3(NT), 0, st, (const f16*)z, ldz, M, C, scale,
                       shift, act, drop, HW, (f16*)y, ldy, amax, nullptr, nullptr, 0.0, nullptr, nullptr);
  else if (ew_wide(amax, true))
    hipLaunchKernelGGL((bn_apply_kernel<float, 1, EW_WIDE>), dim3(wide_grid(total, 256)), dim3(EW_WIDE), 0, st,
                       (const float*)z, ldz, M, C, scale, shift, act, drop, HW, (float*)y, ldy, amax);
  else
    hipLaunchKernelGGL((ew_unroll() == 4 ? bn_apply_kernel<float, 4> : ew_unroll() == 2 ? bn_apply_kernel<float, 2> : bn_apply_kernel<float, 1>), dim3(cs_grid(total)), dim3(NT), 0, st, (const float*)z, ldz, M, C,
                       scale, shift, act, drop, HW, (float*)y, ldy, amax, nullptr, nullptr, 0.0, nullptr, nullptr);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// dg_bn_apply (f32, no dropout) that also writes the f16 x3 pair image of y for the next conv
// (bn_apply_kernel PAIR; include/dgvcc.h)
extern "C" int dg_bn_apply_pair(const float* z, int64_t ldz, int M, int C, const float* scale, const float* shift,
                                const float* mean, const float* invstd, double count, int act, float* y,
                                int64_t ldy, float* amax, void* pair, float* pbound, void* stream) {
  DG_REQUIRE(z && y && scale && shift && mean && invstd && pair && pbound && M > 0 && C > 0 && count >= 1.0);
  DG_REQUIRE(ldz >= C && ldy >= C && (act == 0 || act == 1));
  DG_SUPPORTED(C % 32 == 0 && C <= 4096 && BN_SHAPE_OK(DG_F32, C, ldz) && BN_SHAPE_OK(DG_F32, C, ldy) &&
               EW_WIDE % (C / 4) == 0);
  hipStream_t st = (hipStream_t)stream;
  { const int zr = zero_amax(amax, true, C, st); if (zr != DG_OK) return zr; }
  const long long total = (long long)M * (C / 4);
  hipLaunchKernelGGL((bn_apply_kernel<float, 1, EW_WIDE, 1>), dim3(wide_grid(total, 256)), dim3(EW_WIDE), 0, st, z, ldz,
                     M, C, scale, shift, act, (const float*)nullptr, 1, y, ldy, amax, mean, invstd, count,
                     (unsigned char*)pair, pbound);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_bn_bwd(int dtype, const void* g, int64_t ldg, const void* z, int64_t ldz, int M, int C,
                         const float* gamma, const float* save_mean, const float* save_invstd, const float* scale,
                         const float* shift, int act, const float* drop, int HW, void* dz, int64_t lddz,
                         float* dgamma, float* dbeta, float* dbias, void* workspace, float* amax, void* stream) {
  DG_REQUIRE(g && z && dz && workspace && M > 0 && C > 0);
  DG_REQUIRE((save_mean && save_invstd && scale && shift) || (!save_mean && !save_invstd));
  DG_REQUIRE(!drop || HW > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(BN_SHAPE_OK(dtype, C, ldg) && BN_SHAPE_OK(dtype, C, ldz) && BN_SHAPE_OK(dtype, C, lddz));
  hipStream_t st = (hipStream_t)stream;
  return dtype == DG_BF16
             ? bn_bwd_impl<bf16>(g, ldg, z, ldz, M, C, gamma, save_mean, save_invstd, scale, shift, act, drop, HW, dz,
                                 lddz, dgamma, dbeta, dbias, workspace, st, nullptr, amax)
             : dtype == DG_F16 ? bn_bwd_impl<f16>(g, ldg, z, ldz, M, C, gamma, save_mean, save_invstd, scale, shift, act, drop, HW, dz,
                                 lddz, dgamma, dbeta, dbias, workspace, st, nullptr, amax) : bn_bwd_impl<float>(g, ldg, z, ldz, M, C, gamma, save_mean, save_invstd, scale, shift, act, drop, HW,
                                  dz, lddz, dgamma, dbeta, dbias, workspace, st, nullptr, amax);
}

// dg_bn_bwd with the partial sums already computed by the producer of g (the dgrad
// epilogue, dg_conv_fwd_bnbwd): finalize + apply.  part[nblk][3][C]; workspace >= 3*C floats.
extern "C" int dg_bn_bwd_from_part(int dtype, const float* part, int nblk, const void* g, int64_t ldg, const void* z,
                                   int64_t ldz, int M, int C, const float* gamma, const float* save_mean,
                                   const float* save_invstd, const float* scale, const float* shift, int act,
                                   const float* drop, int HW, void* dz, int64_t lddz, float* dgamma, float* dbeta,
                                   float* dbias, float* coef, float* amax, void* stream) {
  DG_REQUIRE(part && nblk > 0 && g && z && dz && coef && save_mean && save_invstd && scale && shift && M > 0 && C > 0);
  DG_REQUIRE(!drop || HW > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(BN_SHAPE_OK(dtype, C, ldg) && BN_SHAPE_OK(dtype, C, ldz) && BN_SHAPE_OK(dtype, C, lddz));
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_bwd_finalize, dim3(dg_cdiv(C, 16)), dim3(NT), 0, st, part, nblk, M, C, gamma, save_invstd,
                     dgamma, dbeta, dbias, coef);
  DG_CHECK_LAUNCH();
  { const int zr = zero_amax(amax, dtype == DG_F32, C, st); if (zr != DG_OK) return zr; }
  if (dtype == DG_BF16) {
    const long long total = (long long)M * (C / 8);
    hipLaunchKernelGGL((ew_unroll() == 2 ? bn_bwd_apply<bf16, 2> : bn_bwd_apply<bf16, 1>), dim3(cs_grid(total)), dim3(NT), 0, st, (const bf16*)g, ldg, (const bf16*)z,
                       ldz, M, C, save_mean, save_invstd, scale, shift, act, drop, HW, coef, (bf16*)dz, lddz, amax, nullptr, 0, nullptr, nullptr);
  } else if (dtype == DG_F16) {
    const long long total = (long long)M * (C / 8);
    hipLaunchKernelGGL((ew_unroll() == 2 ? bn_bwd_apply<f16, 2> : bn_bwd_apply<f16, 1>), dim3(cs_grid(total)), dim3(NT), 0, st, (const f16*)g, ldg, (const f16*)z,
                       ldz, M, C, save_mean, save_invstd, scale, shift, act, drop, HW, coef, (f16*)dz, lddz, amax, nullptr, 0, nullptr, nullptr);
  } else if (ew_wide(amax, true)) {
    const long long total = (long long)M * (C / 4);
    hipLaunchKernelGGL((bn_bwd_apply<float, 1, EW_WIDE>), dim3(wide_grid(total, 256)), dim3(EW_WIDE), 0, st,
                       (const float*)g, ldg, (const float*)z, ldz, M, C, save_mean, save_invstd, scale, shift, act,
                       drop, HW, coef, (float*)dz, lddz, amax);
  } else {
    const long long total = (long long)M * (C / 4);
    hipLaunchKernelGGL((ew_unroll() == 2 ? bn_bwd_apply<float, 2> : bn_bwd_apply<float, 1>), dim3(cs_grid(total)), dim3(NT), 0, st, (const float*)g, ldg,
                       (const float*)z, ldz, M, C, save_mean, save_invstd, scale, shift, act, drop, HW, coef,
                       (float*)dz, lddz, amax, nullptr, 0, nullptr, nullptr);
  }
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// bn_bwd_finalize on caller-made partial sums part[nblk][3][C] (sum g', sum g' xhat,
// sum xhat): the BN-backward coefficients coef[3][C] and dgamma/dbeta/dbias.
extern "C" int dg_bn_bwd_finalize_part(const float* part, int nblk, int M, int C, const float* gamma,
                                       const float* save_invstd, float* dgamma, float* dbeta, float* dbias,
                                       float* coef, void* stream) {
  DG_REQUIRE(part && nblk > 0 && M > 0 && C > 0 && save_invstd && coef);
  hipLaunchKernelGGL(bn_bwd_finalize, dim3(dg_cdiv(C, 16)), dim3(NT), 0, (hipStream_t)stream, part, nblk, M, C,
                     gamma, save_invstd, dgamma, dbeta, dbias, coef);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_bn_bwd_coef(int dtype, const void* g, int64_t ldg, const void* z, int64_t ldz, int M, int C,
                              const float* gamma, const float* save_mean, const float* save_invstd,
                              const float* scale, const float* shift, int act, const float* drop, int HW,
                              float* coef, float* dgamma, float* dbeta, float* dbias, void* workspace,
                              void* stream) {
  DG_REQUIRE(g && z && coef && workspace && save_mean && save_invstd && scale && shift && M > 0 && C > 0);
  DG_REQUIRE(!drop || HW > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(BN_SHAPE_OK(dtype, C, ldg) && BN_SHAPE_OK(dtype, C, ldz));
  hipStream_t st = (hipStream_t)stream;
  return dtype == DG_BF16
             ? bn_bwd_impl<bf16>(g, ldg, z, ldz, M, C, gamma, save_mean, save_invstd, scale, shift, act, drop, HW,
                                 nullptr, 0, dgamma, dbeta, dbias, workspace, st, coef)
             : dtype == DG_F16 ? bn_bwd_impl<f16>(g, ldg, z, ldz, M, C, gamma, save_mean, save_invstd, scale, shift, act, drop, HW,
                                 nullptr, 0, dgamma, dbeta, dbias, workspace, st, coef) : bn_bwd_impl<float>(g, ldg, z, ldz, M, C, gamma, save_mean, save_invstd, scale, shift, act, drop, HW,
                                  nullptr, 0, dgamma, dbeta, dbias, workspace, st, coef);
}

extern "C" int dg_bn_apply_pool(int dtype, const void* z, int64_t ldz, int N, int H, int W, int C,
                                const float* scale, const float* shift, int act, const float* drop, void* y,
                                int64_t ldy, void* yp, int64_t ldyp, float* amax, void* stream) {
  DG_REQUIRE(z && yp && scale && shift && N > 0 && H > 1 && W > 1 && C > 0 && (act == 0 || act == 1));
  DG_REQUIRE(ldz >= C && ldyp >= C && (!y || ldy >= C));
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(H % 2 == 0 && W % 2 == 0 && (long long)N * H * W < (1LL << 31) && BN_SHAPE_OK(dtype, C, ldz) &&
               BN_SHAPE_OK(dtype, C, ldyp) && (!y || BN_SHAPE_OK(dtype, C, ldy)));
  hipStream_t st = (hipStream_t)stream;
  { const int zr = zero_amax(amax, dtype == DG_F32, C, st); if (zr != DG_OK) return zr; }
  const long long Mp = (long long)N * (H / 2) * (W / 2);
  const long long total = Mp * (C / (DG_IS16(dtype) ? 8 : 4));
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(bn_apply_pool_kernel<bf16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const bf16*)z, ldz, H, W,
                       Mp, C, scale, shift, act, drop, H * W, (bf16*)y, ldy, (bf16*)yp, ldyp, amax);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(bn_apply_pool_kernel<f16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const f16*)z, ldz, H, W,
                       Mp, C, scale, shift, act, drop, H * W, (f16*)y, ldy, (f16*)yp, ldyp, amax);
  else if (ew_wide(amax, true))
    hipLaunchKernelGGL((bn_apply_pool_kernel<float, EW_WIDE>), dim3(wide_grid(total, 512)), dim3(EW_WIDE), 0, st,
                       (const float*)z, ldz, H, W, Mp, C, scale, shift, act, drop, H * W, (float*)y, ldy, (float*)yp,
                       ldyp, amax);
  else
    hipLaunchKernelGGL(bn_apply_pool_kernel<float>, dim3(ew_grid(total)), dim3(NT), 0, st, (const float*)z, ldz, H,
                       W, Mp, C, scale, shift, act, drop, H * W, (float*)y, ldy, (float*)yp, ldyp, amax);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// dg_bn_bwd (f32, train-mode statistics over count pixels, no dropout) that also writes the f16 x3 pair
// image of dz for the dgrad (include/dgvcc.h): bn_bwd_partial's max |g'| rows -> bn_bwd_finalize's bound
// partials -> bn_bwd_apply PAIR
extern "C" int dg_bn_bwd_pair(const float* g, int64_t ldg, const float* z, int64_t ldz, int M, int C,
                              const float* gamma, const float* save_mean, const float* save_invstd,
                              const float* scale, const float* shift, int act, double count, float* dz,
                              int64_t lddz, float* dgamma, float* dbeta, float* dbias, void* workspace, float* amax,
                              void* pair, float* pbound, void* stream) {
  DG_REQUIRE(g && z && dz && workspace && save_mean && save_invstd && scale && shift && pair && pbound && M > 0 &&
             C > 0 && count >= 1.0 && (act == 0 || act == 1));
  DG_SUPPORTED(C % 32 == 0 && C <= 4096 && EW_WIDE % (C / 4) == 0 && BN_SHAPE_OK(DG_F32, C, ldg) &&
               BN_SHAPE_OK(DG_F32, C, ldz) && BN_SHAPE_OK(DG_F32, C, lddz));
  hipStream_t st = (hipStream_t)stream;
  const int nblk = bn_nblk(M);
  const int ppb = dg_cdiv(M, nblk);
  float* part = (float*)workspace;
  float* coef = part + (long long)nblk * 3 * C;
  float* gpart = coef + 3 * C;
  float* bpart = gpart + (long long)nblk * C;
  hipLaunchKernelGGL(bn_bwd_partial<float>, dim3(nblk), dim3(NT), 0, st, g, ldg, z, ldz, M, C, ppb, save_mean,
                     save_invstd, scale, shift, act, (const float*)nullptr, 1, part, gpart);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_bwd_finalize, dim3(dg_cdiv(C, 16)), dim3(NT), 0, st, part, nblk, M, C, gamma, save_invstd,
                     dgamma, dbeta, dbias, coef, gpart, bpart, count);
  DG_CHECK_LAUNCH();
  { const int zr = zero_amax(amax, true, C, st); if (zr != DG_OK) return zr; }
  const long long total = (long long)M * (C / 4);
  hipLaunchKernelGGL((bn_bwd_apply<float, 1, EW_WIDE, 1>), dim3(wide_grid(total, 256)), dim3(EW_WIDE), 0, st, g, ldg,
                     z, ldz, M, C, save_mean, save_invstd, scale, shift, act, (const float*)nullptr, 1, coef, dz, lddz,
                     amax, bpart, dg_cdiv(C, 16), (unsigned char*)pair, pbound);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// dg_bn_bwd_pool (f32, no dropout) with the pair image of dz (as dg_bn_bwd_pair)
extern "C" int dg_bn_bwd_pool_pair(const float* gp, int64_t ldgp, const float* gd, int64_t ldgd, const float* z,
                                   int64_t ldz, int N, int H, int W, int C, const float* gamma, const float* save_mean,
                                   const float* save_invstd, const float* scale, const float* shift, int act,
                                   double count, float* dz, int64_t lddz, float* dgamma, float* dbeta, float* dbias,
                                   void* workspace, float* amax, void* pair, float* pbound, void* stream) {
  DG_REQUIRE(gp && z && dz && workspace && save_mean && save_invstd && scale && shift && pair && pbound);
  DG_REQUIRE(N > 0 && H > 1 && W > 1 && C > 0 && count >= 1.0 && (act == 0 || act == 1));
  DG_SUPPORTED(H % 2 == 0 && W % 2 == 0 && (long long)N * H * W < (1LL << 31) && C % 32 == 0 && C <= 4096 &&
               EW_WIDE % (C / POOL_V) == 0 && BN_SHAPE_OK(DG_F32, C, ldgp) && BN_SHAPE_OK(DG_F32, C, ldz) &&
               BN_SHAPE_OK(DG_F32, C, lddz) && (!gd || BN_SHAPE_OK(DG_F32, C, ldgd)) && NT % (C / POOL_V) == 0);
  hipStream_t st = (hipStream_t)stream;
  const long long M = (long long)N * H * W, Mp = M / 4;
  const int nblk = pool_nblk(Mp);
  const long long ppb = (Mp + nblk - 1) / nblk;
  float* part = (float*)workspace;
  float* coef = part + (long long)nblk * 3 * C;
  float* gpart = coef + 3 * C;
  float* bpart = gpart + (long long)nblk * C;
  hipLaunchKernelGGL(bn_pool_bwd_partial<float>, dim3(nblk), dim3(NT), 0, st, gp, ldgp, gd, ldgd, z, ldz, H, W, Mp, C,
                     ppb, save_mean, save_invstd, scale, shift, act, (const float*)nullptr, H * W, part, gpart);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_bwd_finalize, dim3(dg_cdiv(C, 16)), dim3(NT), 0, st, part, nblk, (int)M, C, gamma, save_invstd,
                     dgamma, dbeta, dbias, coef, gpart, bpart, count);
  DG_CHECK_LAUNCH();
  { const int zr = zero_amax(amax, true, C, st); if (zr != DG_OK) return zr; }
  const long long total = Mp * (C / POOL_V);
  hipLaunchKernelGGL((bn_pool_bwd_apply<float, EW_WIDE, 1>), dim3(wide_grid(total, 512)), dim3(EW_WIDE), 0, st, gp,
                     ldgp, gd, ldgd, z, ldz, H, W, Mp, C, save_mean, save_invstd, scale, shift, act,
                     (const float*)nullptr, H * W, coef, dz, lddz, amax, bpart, dg_cdiv(C, 16), (unsigned char*)pair,
                     pbound);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// dg_bn_apply_pool (f32, no dropout) that also writes the f16 x3 pair image of yp (include/dgvcc.h)
extern "C" int dg_bn_apply_pool_pair(const float* z, int64_t ldz, int N, int H, int W, int C, const float* scale,
                                     const float* shift, const float* mean, const float* invstd, double count,
                                     int act, float* y, int64_t ldy, float* yp, int64_t ldyp, float* amax,
                                     void* pair, float* pbound, void* stream) {
  DG_REQUIRE(z && yp && scale && shift && mean && invstd && pair && pbound && N > 0 && H > 1 && W > 1 && C > 0);
  DG_REQUIRE(count >= 1.0 && (act == 0 || act == 1) && ldz >= C && ldyp >= C && (!y || ldy >= C));
  DG_SUPPORTED(H % 2 == 0 && W % 2 == 0 && (long long)N * H * W < (1LL << 31) && C % 32 == 0 && C <= 4096 &&
               BN_SHAPE_OK(DG_F32, C, ldz) && BN_SHAPE_OK(DG_F32, C, ldyp) && (!y || BN_SHAPE_OK(DG_F32, C, ldy)) &&
               EW_WIDE % (C / 4) == 0);
  hipStream_t st = (hipStream_t)stream;
  { const int zr = zero_amax(amax, true, C, st); if (zr != DG_OK) return zr; }
  const long long Mp = (long long)N * (H / 2) * (W / 2);
  const long long total = Mp * (C / 4);
  hipLaunchKernelGGL((bn_apply_pool_kernel<float, EW_WIDE, 1>), dim3(wide_grid(total, 512)), dim3(EW_WIDE), 0, st, z,
                     ldz, H, W, Mp, C, scale, shift, act, (const float*)nullptr, H * W, y, ldy, yp, ldyp, amax, mean,
                     invstd, count, (unsigned char*)pair, pbound);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

template <typename T>
static int bn_pool_bwd_impl(const void* gp, long long ldgp, const void* gd, long long ldgd, const void* z,
                            long long ldz, int N, int H, int W, int C, const float* gamma, const float* mean,
                            const float* inv, const float* scale, const float* shift, int act, const float* drop,
                            void* dz, long long lddz, float* dgamma, float* dbeta, float* dbias, void* ws,
                            hipStream_t st, float* amax = nullptr) {
  const long long M = (long long)N * H * W, Mp = M / 4;
  const int nblk = pool_nblk(Mp);
  const long long ppb = (Mp + nblk - 1) / nblk;
  float* part = (float*)ws;
  float* coef = part + (long long)nblk * 3 * C;
  hipLaunchKernelGGL(bn_pool_bwd_partial<T>, dim3(nblk), dim3(NT), 0, st, (const T*)gp, ldgp, (const T*)gd, ldgd,
                     (const T*)z, ldz, H, W, Mp, C, ppb, mean, inv, scale, shift, act, drop, H * W, part);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_bwd_finalize, dim3(dg_cdiv(C, 16)), dim3(NT), 0, st, part, nblk, (int)M, C, gamma, inv,
                     dgamma, dbeta, dbias, coef);
  DG_CHECK_LAUNCH();
  const long long total = Mp * (C / POOL_V);
  { const int zr = zero_amax(amax, sizeof(T) == 4, C, st); if (zr != DG_OK) return zr; }
  if (ew_wide(amax, sizeof(T) == 4))
    hipLaunchKernelGGL((bn_pool_bwd_apply<T, EW_WIDE>), dim3(wide_grid(total, 512)), dim3(EW_WIDE), 0, st, (const T*)gp,
                       ldgp, (const T*)gd, ldgd, (const T*)z, ldz, H, W, Mp, C, mean, inv, scale, shift, act, drop,
                       H * W, coef, (T*)dz, lddz, amax);
  else
    hipLaunchKernelGGL(bn_pool_bwd_apply<T>, dim3(ew_grid(total)), dim3(NT), 0, st, (const T*)gp, ldgp, (const T*)gd,
                       ldgd, (const T*)z, ldz, H, W, Mp, C, mean, inv, scale, shift, act, drop, H * W, coef, (T*)dz,
                       lddz, amax);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_bn_bwd_pool(int dtype, const void* gp, int64_t ldgp, const void* gd, int64_t ldgd, const void* z,
                              int64_t ldz, int N, int H, int W, int C, const float* gamma, const float* save_mean,
                              const float* save_invstd, const float* scale, const float* shift, int act,
                              const float* drop, void* dz, int64_t lddz, float* dgamma, float* dbeta, float* dbias,
                              void* workspace, float* amax, void* stream) {
  DG_REQUIRE(gp && z && dz && workspace && save_mean && save_invstd && scale && shift);
  DG_REQUIRE(N > 0 && H > 1 && W > 1 && C > 0 && (act == 0 || act == 1));
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(H % 2 == 0 && W % 2 == 0 && (long long)N * H * W < (1LL << 31) && BN_SHAPE_OK(dtype, C, ldgp) &&
               BN_SHAPE_OK(dtype, C, ldz) && BN_SHAPE_OK(dtype, C, lddz) && (!gd || BN_SHAPE_OK(dtype, C, ldgd)) &&
               C % POOL_V == 0 && NT % (C / POOL_V) == 0);
  hipStream_t st = (hipStream_t)stream;
  return dtype == DG_BF16
             ? bn_pool_bwd_impl<bf16>(gp, ldgp, gd, ldgd, z, ldz, N, H, W, C, gamma, save_mean, save_invstd, scale,
                                      shift, act, drop, dz, lddz, dgamma, dbeta, dbias, workspace, st, amax)
             : dtype == DG_F16 ? bn_pool_bwd_impl<f16>(gp, ldgp, gd, ldgd, z, ldz, N, H, W, C, gamma, save_mean, save_invstd, scale,
                                      shift, act, drop, dz, lddz, dgamma, dbeta, dbias, workspace, st, amax) : bn_pool_bwd_impl<float>(gp, ldgp, gd, ldgd, z, ldz, N, H, W, C, gamma, save_mean, save_invstd, scale,
                                       shift, act, drop, dz, lddz, dgamma, dbeta, dbias, workspace, st, amax);
}

// ---------------------------------------------------------------------------
// SyncBatchNorm phases (nn.SyncBatchNorm over data-parallel ranks; models/ISW/mynn.py:8-14):
// the host all-gathers / all-reduces the per-rank rows between them (dgvcc_amd/syncbn.py).
// ---------------------------------------------------------------------------
extern "C" int dg_bn_stats_row(int dtype, const void* z, int64_t ldz, int M, int C, float* row, void* workspace,
                               void* stream) {
  DG_REQUIRE(z && row && workspace && M > 0 && C > 0 && ldz >= C);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(BN_SHAPE_OK(dtype, C, ldz));
  hipStream_t st = (hipStream_t)stream;
  const int nblk = bn_nblk(M);
  const int ppb = dg_cdiv(M, nblk);
  float* part = (float*)workspace;
  if (dtype == DG_BF16) {
    hipLaunchKernelGGL(bn_stats_partial<bf16>, dim3(nblk), dim3(NT), 0, st, (const bf16*)z, ldz, M, C, ppb, part);
    hipLaunchKernelGGL((bn_stats_finalize<bf16, true>), dim3(dg_cdiv(C, 16)), dim3(NT), 0, st, (const bf16*)z,
                       (const float*)part, nblk, M, C, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, row, nullptr,
                       nullptr, nullptr);
  } else if (dtype == DG_F16) {
    hipLaunchKernelGGL(bn_stats_partial<f16>, dim3(nblk), dim3(NT), 0, st, (const f16*)z, ldz, M, C, ppb, part);
    hipLaunchKernelGGL((bn_stats_finalize<f16, true>), dim3(dg_cdiv(C, 16)), dim3(NT), 0, st, (const f16*)z,
                       (const float*)part, nblk, M, C, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, row, nullptr,
                       nullptr, nullptr);
  } else {
    hipLaunchKernelGGL(bn_stats_partial<float>, dim3(nblk), dim3(NT), 0, st, (const float*)z, ldz, M, C, ppb, part);
    hipLaunchKernelGGL((bn_stats_finalize<float, true>), dim3(dg_cdiv(C, 16)), dim3(NT), 0, st, (const float*)z,
                       (const float*)part, nblk, M, C, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, row, nullptr,
                       nullptr, nullptr);
  }
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_bn_part_sums(const float* part, int nblk, int C, float* sums, void* stream) {
  DG_REQUIRE(part && sums && nblk > 0 && C > 0);
  hipLaunchKernelGGL(bn_sum_rows3, dim3(dg_cdiv(C, 16)), dim3(NT), 0, (hipStream_t)stream, part, nblk, C, sums);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_bn_bwd_sums(int dtype, const void* g, int64_t ldg, const void* z, int64_t ldz, int M, int C,
                              const float* save_mean, const float* save_invstd, const float* scale,
                              const float* shift, int act, const float* drop, int HW, float* sums, void* workspace,
                              void* stream) {
  DG_REQUIRE(g && z && sums && workspace && save_mean && save_invstd && scale && shift && M > 0 && C > 0);
  DG_REQUIRE(!drop || HW > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(BN_SHAPE_OK(dtype, C, ldg) && BN_SHAPE_OK(dtype, C, ldz));
  hipStream_t st = (hipStream_t)stream;
  const int nblk = bn_nblk(M);
  const int ppb = dg_cdiv(M, nblk);
  float* part = (float*)workspace;
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(bn_bwd_partial<bf16>, dim3(nblk), dim3(NT), 0, st, (const bf16*)g, ldg, (const bf16*)z, ldz, M,
                       C, ppb, save_mean, save_invstd, scale, shift, act, drop, HW, part);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(bn_bwd_partial<f16>, dim3(nblk), dim3(NT), 0, st, (const f16*)g, ldg, (const f16*)z, ldz, M,
                       C, ppb, save_mean, save_invstd, scale, shift, act, drop, HW, part);
  else
    hipLaunchKernelGGL(bn_bwd_partial<float>, dim3(nblk), dim3(NT), 0, st, (const float*)g, ldg, (const float*)z,
                       ldz, M, C, ppb, save_mean, save_invstd, scale, shift, act, drop, HW, part);
  DG_CHECK_LAUNCH();
  return dg_bn_part_sums(part, nblk, C, sums, stream);
}

extern "C" int dg_bn_bwd_pool_sums(int dtype, const void* gp, int64_t ldgp, const void* gd, int64_t ldgd,
                                   const void* z, int64_t ldz, int N, int H, int W, int C, const float* save_mean,
                                   const float* save_invstd, const float* scale, const float* shift, int act,
                                   const float* drop, float* sums, void* workspace, void* stream) {
  DG_REQUIRE(gp && z && sums && workspace && save_mean && save_invstd && scale && shift);
  DG_REQUIRE(N > 0 && H > 1 && W > 1 && C > 0 && (act == 0 || act == 1));
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(H % 2 == 0 && W % 2 == 0 && (long long)N * H * W < (1LL << 31) && BN_SHAPE_OK(dtype, C, ldgp) &&
               BN_SHAPE_OK(dtype, C, ldz) && (!gd || BN_SHAPE_OK(dtype, C, ldgd)) && C % POOL_V == 0 &&
               NT % (C / POOL_V) == 0);
  hipStream_t st = (hipStream_t)stream;
  const long long Mp = (long long)N * (H / 2) * (W / 2);
  const int nblk = pool_nblk(Mp);
  const long long ppb = (Mp + nblk - 1) / nblk;
  float* part = (float*)workspace;
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(bn_pool_bwd_partial<bf16>, dim3(nblk), dim3(NT), 0, st, (const bf16*)gp, ldgp, (const bf16*)gd,
                       ldgd, (const bf16*)z, ldz, H, W, Mp, C, ppb, save_mean, save_invstd, scale, shift, act, drop,
                       H * W, part);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(bn_pool_bwd_partial<f16>, dim3(nblk), dim3(NT), 0, st, (const f16*)gp, ldgp, (const f16*)gd,
                       ldgd, (const f16*)z, ldz, H, W, Mp, C, ppb, save_mean, save_invstd, scale, shift, act, drop,
                       H * W, part);
  else
    hipLaunchKernelGGL(bn_pool_bwd_partial<float>, dim3(nblk), dim3(NT), 0, st, (const float*)gp, ldgp,
                       (const float*)gd, ldgd, (const float*)z, ldz, H, W, Mp, C, ppb, save_mean, save_invstd, scale,
                       shift, act, drop, H * W, part);
  DG_CHECK_LAUNCH();
  return dg_bn_part_sums(part, nblk, C, sums, stream);
}

extern "C" int dg_bn_bwd_finalize_sync(const float* sums_local, const float* sums_global, int M_local,
                                       int64_t M_global, int C, const float* gamma, const float* save_invstd,
                                       float* dgamma, float* dbeta, float* dbias, float* coef, void* stream) {
  DG_REQUIRE(sums_local && sums_global && save_invstd && coef && M_local > 0 && C > 0);
  DG_REQUIRE(M_global <= 0 || M_global >= M_local);  // <= 0: read from sums_global's fourth row (C >= 2)
  DG_REQUIRE(M_global > 0 || C >= 2);
  hipLaunchKernelGGL(bn_bwd_finalize_sync, dim3(dg_cdiv(C, NT)), dim3(NT), 0, (hipStream_t)stream, sums_local,
                     sums_global, M_local, (double)M_global, C, gamma, save_invstd, dgamma, dbeta, dbias, coef);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_bn_bwd_apply_coef(int dtype, const void* g, int64_t ldg, const void* z, int64_t ldz, int M, int C,
                                    const float* save_mean, const float* save_invstd, const float* scale,
                                    const float* shift, int act, const float* drop, int HW, const float* coef,
                                    void* dz, int64_t lddz, float* amax, void* stream) {
  DG_REQUIRE(g && z && dz && coef && save_mean && save_invstd && scale && shift && M > 0 && C > 0);
  DG_REQUIRE(!drop || HW > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(BN_SHAPE_OK(dtype, C, ldg) && BN_SHAPE_OK(dtype, C, ldz) && BN_SHAPE_OK(dtype, C, lddz));
  hipStream_t st = (hipStream_t)stream;
  { const int zr = zero_amax(amax, dtype == DG_F32, C, st); if (zr != DG_OK) return zr; }
  const long long total = (long long)M * (C / (DG_IS16(dtype) ? 8 : 4));
  if (dtype == DG_BF16)
    hipLaunchKernelGGL((ew_unroll() == 2 ? bn_bwd_apply<bf16, 2> : bn_bwd_apply<bf16, 1>), dim3(cs_grid(total)), dim3(NT), 0, st, (const bf16*)g, ldg, (const bf16*)z,
                       ldz, M, C, save_mean, save_invstd, scale, shift, act, drop, HW, coef, (bf16*)dz, lddz, amax, nullptr, 0, nullptr, nullptr);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL((ew_unroll() == 2 ? bn_bwd_apply<f16, 2> : bn_bwd_apply<f16, 1>), dim3(cs_grid(total)), dim3(NT), 0, st, (const f16*)g, ldg, (const f16*)z,
                       ldz, M, C, save_mean, save_invstd, scale, shift, act, drop, HW, coef, (f16*)dz, lddz, amax, nullptr, 0, nullptr, nullptr);
  else if (ew_wide(amax, true))
    hipLaunchKernelGGL((bn_bwd_apply<float, 1, EW_WIDE>), dim3(wide_grid(total, 256)), dim3(EW_WIDE), 0, st,
                       (const float*)g, ldg, (const float*)z, ldz, M, C, save_mean, save_invstd, scale, shift, act,
                       drop, HW, coef, (float*)dz, lddz, amax);
  else
    hipLaunchKernelGGL((ew_unroll() == 2 ? bn_bwd_apply<float, 2> : bn_bwd_apply<float, 1>), dim3(cs_grid(total)), dim3(NT), 0, st, (const float*)g, ldg,
                       (const float*)z, ldz, M, C, save_mean, save_invstd, scale, shift, act, drop, HW, coef,
                       (float*)dz, lddz, amax, nullptr, 0, nullptr, nullptr);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_bn_bwd_pool_apply_coef(int dtype, const void* gp, int64_t ldgp, const void* gd, int64_t ldgd,
                                         const void* z, int64_t ldz, int N, int H, int W, int C,
                                         const float* save_mean, const float* save_invstd, const float* scale,
                                         const float* shift, int act, const float* drop, const float* coef, void* dz,
                                         int64_t lddz, float* amax, void* stream) {
  DG_REQUIRE(gp && z && dz && coef && save_mean && save_invstd && scale && shift);
  DG_REQUIRE(N > 0 && H > 1 && W > 1 && C > 0 && (act == 0 || act == 1));
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(H % 2 == 0 && W % 2 == 0 && (long long)N * H * W < (1LL << 31) && BN_SHAPE_OK(dtype, C, ldgp) &&
               BN_SHAPE_OK(dtype, C, ldz) && BN_SHAPE_OK(dtype, C, lddz) && (!gd || BN_SHAPE_OK(dtype, C, ldgd)) &&
               C % POOL_V == 0 && NT % (C / POOL_V) == 0);
  hipStream_t st = (hipStream_t)stream;
  const long long Mp = (long long)N * (H / 2) * (W / 2);
  const long long total = Mp * (C / POOL_V);
  { const int zr = zero_amax(amax, dtype == DG_F32, C, st); if (zr != DG_OK) return zr; }
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(bn_pool_bwd_apply<bf16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const bf16*)gp, ldgp,
                       (const bf16*)gd, ldgd, (const bf16*)z, ldz, H, W, Mp, C, save_mean, save_invstd, scale, shift,
                       act, drop, H * W, coef, (bf16*)dz, lddz, amax);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(bn_pool_bwd_apply<f16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const f16*)gp, ldgp,
                       (const f16*)gd, ldgd, (const f16*)z, ldz, H, W, Mp, C, save_mean, save_invstd, scale, shift,
                       act, drop, H * W, coef, (f16*)dz, lddz, amax);
  else if (ew_wide(amax, true))
    hipLaunchKernelGGL((bn_pool_bwd_apply<float, EW_WIDE>), dim3(wide_grid(total, 512)), dim3(EW_WIDE), 0, st,
                       (const float*)gp, ldgp, (const float*)gd, ldgd, (const float*)z, ldz, H, W, Mp, C, save_mean,
                       save_invstd, scale, shift, act, drop, H * W, coef, (float*)dz, lddz, amax);
  else
    hipLaunchKernelGGL(bn_pool_bwd_apply<float>, dim3(ew_grid(total)), dim3(NT), 0, st, (const float*)gp, ldgp,
                       (const float*)gd, ldgd, (const float*)z, ldz, H, W, Mp, C, save_mean, save_invstd, scale,
                       shift, act, drop, H * W, coef, (float*)dz, lddz, amax);
  DG_CHECK_LAUNCH();
  return DG_OK;
}
