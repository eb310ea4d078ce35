// Max-pool 2x2/2 and bilinear / nearest upsampling on NHWC activations.
//   nn.MaxPool2d(2, 2)       — vgg16_bn.features[6,13,23,33] (models/models.py:35-38)
//   F.interpolate(...)        — upsample() (models/models.py:23-27), cls-map
//                               nearest x4 (models/models.py:200-207),
//                               nn.UpsamplingBilinear2d (align_corners=True,
//                               models/ISW/__init__.py:46, models/SW/__init__.py:37)
// Index/weight rules follow ATen's upsample kernels: align_corners=False uses
// src = (dst + 0.5) / scale - 0.5 clamped at 0; nearest uses floor(dst / scale).
// The backward is a deterministic gather (no atomics).
#include "dg_common.h"
#include <algorithm>

namespace {

constexpr int NT = 256;

inline int ew_grid(long long n) {
  long long g = (n + NT - 1) / NT;
  return (int)std::max<long long>(1, std::min<long long>(g, 16384));
}

// first-max with NaN propagation, scan order (0,0),(0,1),(1,0),(1,1) as ATen
__device__ __forceinline__ int argmax4(float a, float b, float c, float d, float& m) {
  int k = 0; m = a;
  if (b > m || isnan(b)) { m = b; k = 1; }
  if (c > m || isnan(c)) { m = c; k = 2; }
  if (d > m || isnan(d)) { m = d; k = 3; }
  return k;
}

template <typename T>
__global__ __launch_bounds__(NT) void maxpool_fwd_kernel(const T* __restrict__ x, long long ldx, int N, int H, int W,
                                                         int C, T* __restrict__ y, long long ldy) {
  constexpr int V = 16 / (int)sizeof(T);
  const int Ho = H / 2, Wo = W / 2, tpp = C / V;
  const long long total = (long long)N * Ho * Wo * tpp;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int ch = (int)(i % tpp);
    long long t = i / tpp;
    const int wo = (int)(t % Wo); t /= Wo;
    const int ho = (int)(t % Ho);
    const int n = (int)(t / Ho);
    const long long p00 = ((long long)n * H + 2 * ho) * W + 2 * wo;
    float a[V], b[V], c[V], d[V], o[V];
    ldv(x + p00 * ldx + ch * V, a);
    ldv(x + (p00 + 1) * ldx + ch * V, b);
    ldv(x + (p00 + W) * ldx + ch * V, c);
    ldv(x + (p00 + W + 1) * ldx + ch * V, d);
#pragma unroll
    for (int e = 0; e < V; ++e) argmax4(a[e], b[e], c[e], d[e], o[e]);
    stv(y + ((long long)(n * Ho + ho) * Wo + wo) * ldy + ch * V, o);
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void maxpool_bwd_kernel(const T* __restrict__ x, long long ldx,
                                                         const T* __restrict__ gy, long long ldgy, int N, int H, int W,
                                                         int C, T* __restrict__ gx, long long ldgx, int accumulate) {
  constexpr int V = 16 / (int)sizeof(T);
  const int Ho = H / 2, Wo = W / 2, tpp = C / V;
  const long long total = (long long)N * Ho * Wo * tpp;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int ch = (int)(i % tpp);
    long long t = i / tpp;
    const int wo = (int)(t % Wo); t /= Wo;
    const int ho = (int)(t % Ho);
    const int n = (int)(t / Ho);
    const long long p00 = ((long long)n * H + 2 * ho) * W + 2 * wo;
    const long long pos[4] = {p00, p00 + 1, p00 + W, p00 + W + 1};
    float xv[4][V], g[V], out[4][V];
#pragma unroll
    for (int k = 0; k < 4; ++k) ldv(x + pos[k] * ldx + ch * V, xv[k]);
    ldv(gy + ((long long)(n * Ho + ho) * Wo + wo) * ldgy + ch * V, g);
    if (accumulate) {
#pragma unroll
      for (int k = 0; k < 4; ++k) ldv(gx + pos[k] * ldgx + ch * V, out[k]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < V; ++e) out[k][e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < V; ++e) {
      float m;
      const int k = argmax4(xv[0][e], xv[1][e], xv[2][e], xv[3][e], m);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
        if (kk == k) out[kk][e] += g[e];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) stv(gx + pos[k] * ldgx + ch * V, out[k]);
  }
}

// General max-pool (ResNet stem: 3x3, stride 2, pad 1; -inf padding, first max
// in (kh, kw) scan order, NaN propagates — ATen max_pool2d).
template <typename T>
__global__ __launch_bounds__(NT) void maxpool_gen_fwd(const T* __restrict__ x, long long ldx, int N, int H, int W, int C,
                                                      int k, int st, int pad, int P, int Q, T* __restrict__ y,
                                                      long long ldy) {
  constexpr int V = 16 / (int)sizeof(T);
  const int tpp = C / V;
  const long long total = (long long)N * P * Q * tpp;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int ch = (int)(i % tpp);
    long long t = i / tpp;
    const int q = (int)(t % Q); t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float m[V];
#pragma unroll
    for (int e = 0; e < V; ++e) m[e] = -INFINITY;
    for (int r = 0; r < k; ++r) {
      const int h = p * st - pad + r;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int s = 0; s < k; ++s) {
        const int w = q * st - pad + s;
        if ((unsigned)w >= (unsigned)W) continue;
        float v[V];
        ldv(x + (((long long)n * H + h) * W + w) * ldx + ch * V, v);
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (v[e] > m[e] || isnan(v[e])) m[e] = v[e];
      }
    }
    stv(y + (((long long)n * P + p) * Q + q) * ldy + ch * V, m);
  }
}

// gather backward: input (h,w) collects gy of every window whose argmax it is
template <typename T>
__global__ __launch_bounds__(NT) void maxpool_gen_bwd(const T* __restrict__ x, long long ldx, const T* __restrict__ gy,
                                                      long long ldgy, int N, int H, int W, int C, int k, int st,
                                                      int pad, int P, int Q, T* __restrict__ gx, long long ldgx,
                                                      int accumulate) {
  constexpr int V = 16 / (int)sizeof(T);
  const int tpp = C / V;
  const long long total = (long long)N * H * W * tpp;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int ch = (int)(i % tpp);
    long long t = i / tpp;
    const int w = (int)(t % W); t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float acc[V];
    if (accumulate) ldv(gx + (((long long)n * H + h) * W + w) * ldgx + ch * V, acc);
    else {
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] = 0.f;
    }
    // windows p with p*st - pad <= h <= p*st - pad + k - 1
    const int plo = max(0, (h + pad - k + st) / st), phi = min(P - 1, (h + pad) / st);
    const int qlo = max(0, (w + pad - k + st) / st), qhi = min(Q - 1, (w + pad) / st);
    for (int p = plo; p <= phi; ++p)
      for (int q = qlo; q <= qhi; ++q) {
        // argmax of window (p, q), per channel, in scan order
        float m[V];
        int am[V];
#pragma unroll
        for (int e = 0; e < V; ++e) { m[e] = -INFINITY; am[e] = -1; }
        for (int r = 0; r < k; ++r) {
          const int hh = p * st - pad + r;
          if ((unsigned)hh >= (unsigned)H) continue;
          for (int s = 0; s < k; ++s) {
            const int ww = q * st - pad + s;
            if ((unsigned)ww >= (unsigned)W) continue;
            float v[V];
            ldv(x + (((long long)n * H + hh) * W + ww) * ldx + ch * V, v);
#pragma unroll
            for (int e = 0; e < V; ++e)
              if (v[e] > m[e] || isnan(v[e]) || am[e] < 0) { m[e] = v[e]; am[e] = hh * W + ww; }
          }
        }
        float g[V];
        ldv(gy + (((long long)n * P + p) * Q + q) * ldgy + ch * V, g);
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (am[e] == h * W + w) acc[e] += g[e];
      }
    stv(gx + (((long long)n * H + h) * W + w) * ldgx + ch * V, acc);
  }
}

// The same pool recording each window's argmax (uint8 offset r*k + s of the first max,
// same scan order and NaN rule): the backward is then a gather of at most ceil(k/st)^2
// (index, gradient) pairs per input instead of re-scanning every overlapping window
// (9 x-loads per window for the ResNet 3x3/2 stem pool).
template <typename T>
__global__ __launch_bounds__(NT) void maxpool_idx_fwd(const T* __restrict__ x, long long ldx, int N, int H, int W,
                                                      int C, int k, int st, int pad, int P, int Q, T* __restrict__ y,
                                                      long long ldy, unsigned char* __restrict__ idx) {
  constexpr int V = 16 / (int)sizeof(T);
  const int tpp = C / V;
  const int total = N * P * Q * tpp;  // < 2^30 (checked by the ABI)
  for (int i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const int ch = i % tpp;
    int t = i / tpp;
    const int q = t % Q; t /= Q;
    const int p = t % P;
    const int n = t / P;
    float m[V];
    int am[V];
#pragma unroll
    for (int e = 0; e < V; ++e) { m[e] = -INFINITY; am[e] = -1; }
    for (int r = 0; r < k; ++r) {
      const int h = p * st - pad + r;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int s = 0; s < k; ++s) {
        const int w = q * st - pad + s;
        if ((unsigned)w >= (unsigned)W) continue;
        float v[V];
        ldv(x + ((long long)(n * H + h) * W + w) * ldx + ch * V, v);
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (v[e] > m[e] || isnan(v[e]) || am[e] < 0) { m[e] = v[e]; am[e] = r * k + s; }
      }
    }
    const long long o = (long long)(n * P + p) * Q + q;
    stv(y + o * ldy + ch * V, m);
    unsigned int pk[V / 4];
#pragma unroll
    for (int e = 0; e < V / 4; ++e)
      pk[e] = (unsigned)am[4 * e] | ((unsigned)am[4 * e + 1] << 8) | ((unsigned)am[4 * e + 2] << 16) |
              ((unsigned)am[4 * e + 3] << 24);
    unsigned int* ip = reinterpret_cast<unsigned int*>(idx + o * C + ch * V);
#pragma unroll
    for (int e = 0; e < V / 4; ++e) ip[e] = pk[e];
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void maxpool_idx_bwd(const unsigned char* __restrict__ idx, const T* __restrict__ gy,
                                                      long long ldgy, int N, int H, int W, int C, int k, int st,
                                                      int pad, int P, int Q, T* __restrict__ gx, long long ldgx,
                                                      int accumulate) {
  constexpr int V = 16 / (int)sizeof(T);
  const int tpp = C / V;
  const int total = N * H * W * tpp;  // < 2^30 (checked by the ABI)
  for (int i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const int ch = i % tpp;
    int t = i / tpp;
    const int w = t % W; t /= W;
    const int h = t % H;
    const int n = t / H;
    float acc[V];
    T* dst = gx + ((long long)(n * H + h) * W + w) * ldgx + ch * V;
    if (accumulate) ldv(dst, acc);
    else {
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] = 0.f;
    }
    const int plo = max(0, (h + pad - k + st) / st), phi = min(P - 1, (h + pad) / st);
    const int qlo = max(0, (w + pad - k + st) / st), qhi = min(Q - 1, (w + pad) / st);
    for (int p = plo; p <= phi; ++p)
      for (int q = qlo; q <= qhi; ++q) {
        const unsigned mine = (unsigned)((h - (p * st - pad)) * k + (w - (q * st - pad)));
        const long long o = (long long)(n * P + p) * Q + q;
        const unsigned int* ip = reinterpret_cast<const unsigned int*>(idx + o * C + ch * V);
        unsigned int pk[V / 4];
#pragma unroll
        for (int e = 0; e < V / 4; ++e) pk[e] = ip[e];
        float g[V];
        ldv(gy + o * ldgy + ch * V, g);
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (((pk[e >> 2] >> (8 * (e & 3))) & 0xffu) == mine) acc[e] += g[e];
      }
    stv(dst, acc);
  }
}

// Source taps of output index o along one axis.
struct Tap { int i0, i1; float l1; };
__device__ __forceinline__ Tap src_tap(int o, int in, int out, int scale, int mode) {
  Tap t;
  if (mode == 2) {  // nearest
    int i = o / scale;
    if (i > in - 1) i = in - 1;
    t.i0 = t.i1 = i; t.l1 = 0.f;
    return t;
  }
  float src;
  if (mode == 1) {  // align_corners=True
    const float r = out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
    src = r * o;
  } else {
    const float r = 1.0f / (float)scale;
    src = r * (o + 0.5f) - 0.5f;
    if (src < 0.f) src = 0.f;
  }
  int i0 = (int)src;
  if (i0 > in - 1) i0 = in - 1;
  t.i0 = i0;
  t.i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  t.l1 = src - (float)i0;
  return t;
}

template <typename T, int V>
__global__ __launch_bounds__(NT) void upsample_fwd_kernel(const T* __restrict__ x, long long ldx, int N, int H, int W,
                                                          int C, int scale, int mode, T* __restrict__ y,
                                                          long long ldy) {
  const int Ho = H * scale, Wo = W * scale, tpp = C / V;
  const long long total = (long long)N * Ho * Wo * tpp;
  const bool small = total < (1LL << 31);
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    int ch, wo, ho, n;
    if (small) {  // 32-bit index math (64-bit division is a long software sequence)
      const int ii = (int)i;
      ch = ii % tpp;
      int t = ii / tpp;
      wo = t % Wo; t /= Wo;
      ho = t % Ho;
      n = t / Ho;
    } else {
      ch = (int)(i % tpp);
      long long t = i / tpp;
      wo = (int)(t % Wo); t /= Wo;
      ho = (int)(t % Ho);
      n = (int)(t / Ho);
    }
    const Tap th = src_tap(ho, H, Ho, scale, mode), tw = src_tap(wo, W, Wo, scale, mode);
    const float h1l = th.l1, h0l = 1.f - th.l1, w1l = tw.l1, w0l = 1.f - tw.l1;
    const T* base = x + (long long)n * H * W * ldx + ch * V;
    float a[V], b[V], c[V], d[V], o[V];
    if constexpr (V == 1) {
      a[0] = to_f(base[((long long)th.i0 * W + tw.i0) * ldx]);
      b[0] = to_f(base[((long long)th.i0 * W + tw.i1) * ldx]);
      c[0] = to_f(base[((long long)th.i1 * W + tw.i0) * ldx]);
      d[0] = to_f(base[((long long)th.i1 * W + tw.i1) * ldx]);
    } else {
      ldv(base + ((long long)th.i0 * W + tw.i0) * ldx, a);
      ldv(base + ((long long)th.i0 * W + tw.i1) * ldx, b);
      ldv(base + ((long long)th.i1 * W + tw.i0) * ldx, c);
      ldv(base + ((long long)th.i1 * W + tw.i1) * ldx, d);
    }
#pragma unroll
    for (int e = 0; e < V; ++e) o[e] = h0l * (w0l * a[e] + w1l * b[e]) + h1l * (w0l * c[e] + w1l * d[e]);
    T* dst = y + ((long long)(n * Ho + ho) * Wo + wo) * ldy + ch * V;
    if constexpr (V == 1) dst[0] = from_f<T>(o[0]);
    else stv(dst, o);
  }
}

// C = 1 maps (the density heads' x4 / the trunks' x16 upsample): 4 consecutive output columns per
// thread, one row tap, one 4-element store (the per-element arithmetic of upsample_fwd_kernel, so the
// values are identical); a channel-per-thread grid spent most of its issue on index math per 4-B store.
template <typename T>
__global__ __launch_bounds__(NT) void upsample_fwd_c1_kernel(const T* __restrict__ x, long long ldx, int N, int H,
                                                             int W, int scale, int mode, T* __restrict__ y) {
  const int Ho = H * scale, Wo = W * scale, q4 = Wo / 4;
  const int total = N * Ho * q4;  // < 2^31 (checked by the launcher)
  for (int i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const int qq = i % q4;
    const int t = i / q4;
    const int ho = t % Ho, n = t / Ho;
    const Tap th = src_tap(ho, H, Ho, scale, mode);
    const float h1l = th.l1, h0l = 1.f - th.l1;
    const T* r0 = x + ((long long)n * H + th.i0) * W * ldx;
    const T* r1 = x + ((long long)n * H + th.i1) * W * ldx;
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const Tap tw = src_tap(qq * 4 + e, W, Wo, scale, mode);
      const float w1l = tw.l1, w0l = 1.f - tw.l1;
      const float a = to_f(r0[tw.i0 * ldx]), b = to_f(r0[tw.i1 * ldx]);
      const float c = to_f(r1[tw.i0 * ldx]), d = to_f(r1[tw.i1 * ldx]);
      o[e] = h0l * (w0l * a + w1l * b) + h1l * (w0l * c + w1l * d);
    }
    st4(y + (long long)t * Wo + qq * 4, o);
  }
}

// Range of output indices whose taps may touch input index i (superset).
__device__ __forceinline__ void out_range(int i, int in, int out, int scale, int mode, int& lo, int& hi) {
  if (mode == 1) {
    const float r = in > 1 ? (float)(out - 1) / (float)(in - 1) : (float)out;
    lo = (int)floorf((i - 1) * r) - 1;
    hi = (int)ceilf((i + 1) * r) + 2;
  } else {
    lo = scale * (i - 1) - 1;
    hi = scale * (i + 2) + 1;
  }
  lo = max(lo, 0);
  hi = min(hi, out);
}

__device__ __forceinline__ float tap_weight(const Tap& t, int i) {
  float w = 0.f;
  if (t.i0 == i) w += 1.f - t.l1;
  if (t.i1 == i) w += t.l1;
  return w;
}

template <typename T, int V>
__global__ __launch_bounds__(NT) void upsample_bwd_kernel(const T* __restrict__ gy, long long ldgy,
                                                          const T* __restrict__ gy2, long long ldgy2, int N, int H,
                                                          int W, int C, int scale, int mode, T* __restrict__ gx,
                                                          long long ldgx, int accumulate) {
  const int Ho = H * scale, Wo = W * scale, tpp = C / V;
  const long long total = (long long)N * H * W * tpp;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int ch = (int)(i % tpp);
    long long t = i / tpp;
    const int iw = (int)(t % W); t /= W;
    const int ih = (int)(t % H);
    const int n = (int)(t / H);
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
    int hlo, hhi, wlo, whi;
    out_range(ih, H, Ho, scale, mode, hlo, hhi);
    out_range(iw, W, Wo, scale, mode, wlo, whi);
    for (int oh = hlo; oh < hhi; ++oh) {
      const float wh = tap_weight(src_tap(oh, H, Ho, scale, mode), ih);
      if (wh == 0.f) continue;
      for (int ow = wlo; ow < whi; ++ow) {
        const Tap tw = src_tap(ow, W, Wo, scale, mode);
        const float ww = tap_weight(tw, iw);
        if (ww == 0.f) continue;
        // ATen's backward applies h-lambda * w-lambda to each grad element
        const float wgt = wh * ww;
        const long long op = (long long)(n * Ho + oh) * Wo + ow;
        float g[V];
        if constexpr (V == 1) g[0] = to_f(gy[op * ldgy + ch]);
        else ldv(gy + op * ldgy + ch * V, g);
        if (gy2) {
          float g2[V];
          if constexpr (V == 1) g2[0] = to_f(gy2[op * ldgy2 + ch]);
          else ldv(gy2 + op * ldgy2 + ch * V, g2);
#pragma unroll
          for (int e = 0; e < V; ++e) g[e] += g2[e];
        }
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] = fmaf(wgt, g[e], acc[e]);
      }
    }
    T* dst = gx + ((long long)(n * H + ih) * W + iw) * ldgx + ch * V;
    if (accumulate) {
      if constexpr (V == 1) acc[0] += to_f(dst[0]);
      else {
        float o[V];
        ldv(dst, o);
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] += o[e];
      }
    }
    if constexpr (V == 1) dst[0] = from_f<T>(acc[0]);
    else stv(dst, acc);
  }
}

// C = 1 bilinear backward (modes 0 / 1), separable: one block per (image, input row ih, tile of TW
// input columns).  The block first sums each output column of the tile's span over the output rows
// that touch ih (their weights wh formed once, in LDS), coalesced along the row, then every thread
// sums its input column's window of those column sums with its ww.  gx = sum_ow ww * (sum_oh wh * g):
// the same terms as upsample_bwd_kernel's flat sum over (oh, ow) of (wh * ww) * g, grouped by column
// (rounding differs at the f32 ulp level; ATen's own backward adds them with atomics in no fixed order).
// The per-pixel form re-derived every (oh, ow) tap of a 36 x 36 window per input pixel for the x16
// align-corners upsample.  Zero weights are skipped, as there (a NaN/Inf gradient where no tap reads
// it is not propagated).
constexpr int UPC1_SPAN = 8192, UPC1_KH = 128;
template <typename T>
__global__ __launch_bounds__(NT) void upsample_bwd_c1_kernel(const T* __restrict__ gy, long long ldgy,
                                                             const T* __restrict__ gy2, long long ldgy2, int N, int H,
                                                             int W, int scale, int mode, int TW, T* __restrict__ gx,
                                                             long long ldgx, int accumulate) {
  __shared__ float wh[UPC1_KH];
  __shared__ float cs[UPC1_SPAN];
  const int Ho = H * scale, Wo = W * scale;
  const int n = blockIdx.y / H, ih = blockIdx.y - n * H;
  const int iw0 = blockIdx.x * TW, iw1 = min(W, iw0 + TW);
  int hlo, hhi, wlo, whi, dummy;
  out_range(ih, H, Ho, scale, mode, hlo, hhi);
  out_range(iw0, W, Wo, scale, mode, wlo, dummy);
  out_range(iw1 - 1, W, Wo, scale, mode, dummy, whi);
  const int KH = min(hhi - hlo, UPC1_KH), span = min(whi - wlo, UPC1_SPAN);  // launcher bounds both
  for (int k = threadIdx.x; k < KH; k += NT) wh[k] = tap_weight(src_tap(hlo + k, H, Ho, scale, mode), ih);
  __syncthreads();
  // out_range is a superset: read only the rows from the first to the last nonzero weight
  int k0 = KH, k1 = -1;
  for (int k = 0; k < KH; ++k)
    if (wh[k] != 0.f) {
      k0 = min(k0, k);
      k1 = k;
    }
  const long long row0 = (long long)n * Ho + hlo;
  for (int j = threadIdx.x; j < span; j += NT) {
    const long long op0 = row0 * Wo + wlo + j;
    float s = 0.f;
#pragma unroll 4
    for (int k = k0; k <= k1; ++k) {
      const long long op = op0 + (long long)k * Wo;
      float g = to_f(gy[op * ldgy]);
      if (gy2) g += to_f(gy2[op * ldgy2]);
      const float w = wh[k];
      s = w != 0.f ? fmaf(w, g, s) : s;
    }
    cs[j] = s;
  }
  __syncthreads();
  for (int iw = iw0 + threadIdx.x; iw < iw1; iw += NT) {
    int lo, hi;
    out_range(iw, W, Wo, scale, mode, lo, hi);
    float acc = 0.f;
    for (int ow = lo; ow < hi; ++ow) {
      const float w = tap_weight(src_tap(ow, W, Wo, scale, mode), iw);
      acc = w != 0.f ? fmaf(w, cs[ow - wlo], acc) : acc;
    }
    T* dst = gx + ((long long)n * H * W + (long long)ih * W + iw) * ldgx;
    if (accumulate) acc += to_f(dst[0]);
    dst[0] = from_f<T>(acc);
  }
}

// den_dec of the DGModel family on the decomposed decoder concatenation
// (models/models.py:84, 89-90):
//   conv1x1(cat[y1, up2(y2), up4(y3)]) = conv1x1(y1; W1) + up2(conv1x1(y2; W2)) + up4(conv1x1(y3; W3))
// since bilinear resampling acts on pixels and the 1x1 conv on channels (both linear).
// z = z1 + up2(z2) + up4(z3) + bias (bilinear, align_corners=False, as upsample_fwd_kernel),
// stored in T, plus the BN statistics partials (n, mean, M2) of the stored values per block
// (per-block shift = the block's first pixel, recomputed by every thread).
template <typename T>
__device__ __forceinline__ void cat_combine_px(const T* z1, long long ldz1, const T* z2, long long ldz2, const T* z3,
                                               long long ldz3, int H, int W, long long p, int c0, const float* bias,
                                               float o[16 / sizeof(T)]) {
  constexpr int V = 16 / (int)sizeof(T);
  const int HW = H * W;  // N*H*W < 2^31 (checked by the ABI)
  const int n = (int)p / HW;
  const int rem = (int)p - n * HW;
  const int ho = rem / W, wo = rem - ho * W;
  ldv(z1 + p * ldz1 + c0, o);
#pragma unroll
  for (int lv = 0; lv < 2; ++lv) {
    const int sc = lv == 0 ? 2 : 4, h = H / sc, w = W / sc;
    const T* zz = lv == 0 ? z2 : z3;
    const long long ld = lv == 0 ? ldz2 : ldz3;
    const Tap th = src_tap(ho, h, H, sc, 0), tw = src_tap(wo, w, W, sc, 0);
    const float h1l = th.l1, h0l = 1.f - th.l1, w1l = tw.l1, w0l = 1.f - tw.l1;
    const T* base = zz + (long long)n * h * w * ld + c0;
    float a[V], b[V], c[V], d[V];
    ldv(base + ((long long)th.i0 * w + tw.i0) * ld, a);
    ldv(base + ((long long)th.i0 * w + tw.i1) * ld, b);
    ldv(base + ((long long)th.i1 * w + tw.i0) * ld, c);
    ldv(base + ((long long)th.i1 * w + tw.i1) * ld, d);
#pragma unroll
    for (int e = 0; e < V; ++e) o[e] += h0l * (w0l * a[e] + w1l * b[e]) + h1l * (w0l * c[e] + w1l * d[e]);
  }
  if (bias) {
#pragma unroll
    for (int e = 0; e < V; ++e) o[e] += bias[c0 + e];
  }
#pragma unroll
  for (int e = 0; e < V; ++e) o[e] = to_f(from_f<T>(o[e]));  // the stored value
}

template <typename T>
__global__ __launch_bounds__(NT) void cat_combine_kernel(const T* z1, long long ldz1,
                                                         const T* __restrict__ z2, long long ldz2,
                                                         const T* __restrict__ z3, long long ldz3, int H, int W,
                                                         long long M, int C, long long ppb,
                                                         const float* __restrict__ bias, T* z, long long ldz,
                                                         float* __restrict__ part) {
  constexpr int V = 16 / (int)sizeof(T);
  __shared__ float sh[2][NT * V];
  __shared__ float shK[NT * V];
  const int tpp = C / V;
  const int rows = NT / tpp;
  const int tid = threadIdx.x;
  const int ch = tid % tpp, pl = tid / tpp;
  const int c0 = ch * V;
  const long long p0 = blockIdx.x * ppb, p1 = min(M, p0 + ppb);
  float K[V], s1[V], s2[V];
#pragma unroll
  for (int e = 0; e < V; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  // per-channel shift = the block's first pixel, computed before any store (z may alias z1)
  if (pl == 0 && p0 < p1) {
    cat_combine_px<T>(z1, ldz1, z2, ldz2, z3, ldz3, H, W, p0, c0, bias, K);
#pragma unroll
    for (int e = 0; e < V; ++e) shK[c0 + e] = K[e];
  }
  __syncthreads();
  if (pl < rows && p0 < p1) {
#pragma unroll
    for (int e = 0; e < V; ++e) K[e] = shK[c0 + e];
    for (long long p = p0 + pl; p < p1; p += rows) {
      float o[V];
      cat_combine_px<T>(z1, ldz1, z2, ldz2, z3, ldz3, H, W, p, c0, bias, o);
      stv(z + p * ldz + c0, o);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const float dd = o[e] - K[e];
        s1[e] += dd;
        s2[e] = fmaf(dd, dd, s2[e]);
      }
    }
  }
  if (pl < rows) {
#pragma unroll
    for (int e = 0; e < V; ++e) { sh[0][pl * C + c0 + e] = s1[e]; sh[1][pl * C + c0 + e] = s2[e]; }
  }
  __syncthreads();
  if (!part) return;
  for (int c = tid; c < C; c += NT) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rows; ++r) { a += sh[0][r * C + c]; b += sh[1][r * C + c]; }
    const float n = (float)max(0LL, p1 - p0);
    float* out = part + (long long)blockIdx.x * 3 * C;
    out[c] = n;
    out[C + c] = n > 0.f ? shK[c] + a / n : 0.f;
    out[2 * C + c] = n > 0.f ? fmaxf(b - a * a / n, 0.f) : 0.f;
  }
}

inline int cat_nblk(long long M) { return (int)std::max(1LL, std::min(1024LL, (M + 63) / 64)); }

template <typename T>
int up_fwd(const void* x, long long ldx, int N, int H, int W, int C, int scale, int mode, void* y, long long ldy,
           hipStream_t st) {
  constexpr int V = 16 / (int)sizeof(T);
  const bool vec = (C % V == 0) && (ldx % V == 0) && (ldy % V == 0);
  const long long total = (long long)N * H * scale * W * scale * (vec ? C / V : C);
  if (C == 1 && ldy == 1 && (W * scale) % 4 == 0 && total < (1LL << 31) && !getenv("DGVCC_UP_C1_OFF"))
    hipLaunchKernelGGL(upsample_fwd_c1_kernel<T>, dim3(ew_grid(total / 4)), dim3(NT), 0, st, (const T*)x, ldx, N, H, W,
                       scale, mode, (T*)y);
  else if (vec)
    hipLaunchKernelGGL((upsample_fwd_kernel<T, V>), dim3(ew_grid(total)), dim3(NT), 0, st, (const T*)x, ldx, N, H, W,
                       C, scale, mode, (T*)y, ldy);
  else
    hipLaunchKernelGGL((upsample_fwd_kernel<T, 1>), dim3(ew_grid(total)), dim3(NT), 0, st, (const T*)x, ldx, N, H, W,
                       C, scale, mode, (T*)y, ldy);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// Specialised backward for bilinear align_corners=False at a compile-time scale SC
// (the decoder's x2 / x4): the output pixels that touch input i lie in the exact window
// [SC*i - SC/2, SC*i + 3*SC/2) (2*SC per axis, checked against the generic tap rule),
// so the per-axis weights are computed once and the gather loop has fixed trip counts.
// Same (oh, ow) accumulation order as upsample_bwd_kernel -> identical results.
template <typename T, int V, int SC>
__global__ __launch_bounds__(NT) void upsample_bwd_bl_kernel(const T* __restrict__ gy, long long ldgy,
                                                             const T* __restrict__ gy2, long long ldgy2, int N, int H,
                                                             int W, int C, T* __restrict__ gx, long long ldgx,
                                                             int accumulate) {
  constexpr int WN = 2 * SC;
  const int Ho = H * SC, Wo = W * SC, tpp = C / V;
  const int total = N * H * W * tpp;  // < 2^31 (checked by the launcher)
  for (int i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const int ch = i % tpp;
    int t = i / tpp;
    const int iw = t % W; t /= W;
    const int ih = t % H;
    const int n = t / H;
    const int oh0 = SC * ih - SC / 2, ow0 = SC * iw - SC / 2;
    float wh[WN], ww[WN];
#pragma unroll
    for (int k = 0; k < WN; ++k) {
      const int oh = oh0 + k, ow = ow0 + k;
      wh[k] = (oh >= 0 && oh < Ho) ? tap_weight(src_tap(oh, H, Ho, SC, 0), ih) : 0.f;
      ww[k] = (ow >= 0 && ow < Wo) ? tap_weight(src_tap(ow, W, Wo, SC, 0), iw) : 0.f;
    }
    float acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0.f;
#pragma unroll
    for (int kh = 0; kh < WN; ++kh) {
      if (wh[kh] == 0.f) continue;
      const long long rowp = (long long)(n * Ho + oh0 + kh) * Wo;
#pragma unroll
      for (int kw = 0; kw < WN; ++kw) {
        if (ww[kw] == 0.f) continue;
        const float wgt = wh[kh] * ww[kw];
        const long long op = rowp + ow0 + kw;
        float g[V];
        ldv(gy + op * ldgy + ch * V, g);
        if (gy2) {
          float g2[V];
          ldv(gy2 + op * ldgy2 + ch * V, g2);
#pragma unroll
          for (int e = 0; e < V; ++e) g[e] += g2[e];
        }
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] = fmaf(wgt, g[e], acc[e]);
      }
    }
    T* dst = gx + ((long long)(n * H + ih) * W + iw) * ldgx + ch * V;
    if (accumulate) {
      float o[V];
      ldv(dst, o);
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] += o[e];
    }
    stv(dst, acc);
  }
}

template <typename T>
int up_bwd(const void* gy, long long ldgy, const void* gy2, long long ldgy2, int N, int H, int W, int C, int scale,
           int mode, void* gx, long long ldgx, int acc, hipStream_t st) {
  constexpr int V = 16 / (int)sizeof(T);
  const bool vec = (C % V == 0) && (ldgy % V == 0) && (ldgx % V == 0) && (!gy2 || ldgy2 % V == 0);
  const long long total = (long long)N * H * W * (vec ? C / V : C);
  int tw = 0;  // upsample_bwd_c1_kernel's input-column tile: the span and row window fit its LDS
  if (C == 1 && mode != 2 && (long long)N * H <= 65535 && !getenv("DGVCC_UP_C1_OFF")) {
    const double rw = mode == 1 ? (W > 1 ? (double)(W * scale - 1) / (W - 1) : (double)W * scale) : scale;
    const double rh = mode == 1 ? (H > 1 ? (double)(H * scale - 1) / (H - 1) : (double)H * scale) : scale;
    if (3.0 * rh + 8.0 <= UPC1_KH)
      for (tw = std::min(W, NT); tw > 0 && (tw + 3.0) * rw + 8.0 > UPC1_SPAN; tw /= 2) {
      }
  }
  if (tw > 0)
    hipLaunchKernelGGL(upsample_bwd_c1_kernel<T>, dim3(dg_cdiv(W, tw), N * H), dim3(NT), 0, st, (const T*)gy, ldgy,
                       (const T*)gy2, ldgy2, N, H, W, scale, mode, tw, (T*)gx, ldgx, acc);
  else if (vec && mode == 0 && (scale == 2 || scale == 4) && total < (1LL << 31) &&
      (long long)N * H * scale * W * scale < (1LL << 31)) {
    if (scale == 2)
      hipLaunchKernelGGL((upsample_bwd_bl_kernel<T, V, 2>), dim3(ew_grid(total)), dim3(NT), 0, st, (const T*)gy, ldgy,
                         (const T*)gy2, ldgy2, N, H, W, C, (T*)gx, ldgx, acc);
    else
      hipLaunchKernelGGL((upsample_bwd_bl_kernel<T, V, 4>), dim3(ew_grid(total)), dim3(NT), 0, st, (const T*)gy, ldgy,
                         (const T*)gy2, ldgy2, N, H, W, C, (T*)gx, ldgx, acc);
  } else if (vec)
    hipLaunchKernelGGL((upsample_bwd_kernel<T, V>), dim3(ew_grid(total)), dim3(NT), 0, st, (const T*)gy, ldgy,
                       (const T*)gy2, ldgy2, N, H, W, C, scale, mode, (T*)gx, ldgx, acc);
  else
    hipLaunchKernelGGL((upsample_bwd_kernel<T, 1>), dim3(ew_grid(total)), dim3(NT), 0, st, (const T*)gy, ldgy,
                       (const T*)gy2, ldgy2, N, H, W, C, scale, mode, (T*)gx, ldgx, acc);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

}  // namespace

extern "C" int dg_maxpool2_fwd(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, void* y,
                               int64_t ldy, void* stream) {
  DG_REQUIRE(x && y && N > 0 && H > 0 && W > 0 && C > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(H % 2 == 0 && W % 2 == 0 && C % V == 0 && ldx % V == 0 && ldy % V == 0);
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)N * (H / 2) * (W / 2) * (C / V);
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<bf16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const bf16*)x, ldx, N, H, W,
                       C, (bf16*)y, ldy);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<f16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const f16*)x, ldx, N, H, W,
                       C, (f16*)y, ldy);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, dim3(ew_grid(total)), dim3(NT), 0, st, (const float*)x, ldx, N, H,
                       W, C, (float*)y, ldy);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_maxpool2_bwd(int dtype, const void* x, int64_t ldx, const void* gy, int64_t ldgy, int N, int H,
                               int W, int C, void* gx, int64_t ldgx, int accumulate, void* stream) {
  DG_REQUIRE(x && gy && gx && N > 0 && H > 0 && W > 0 && C > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(H % 2 == 0 && W % 2 == 0 && C % V == 0 && ldx % V == 0 && ldgy % V == 0 && ldgx % V == 0);
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)N * (H / 2) * (W / 2) * (C / V);
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<bf16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const bf16*)x, ldx,
                       (const bf16*)gy, ldgy, N, H, W, C, (bf16*)gx, ldgx, accumulate);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<f16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const f16*)x, ldx,
                       (const f16*)gy, ldgy, N, H, W, C, (f16*)gx, ldgx, accumulate);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<float>, dim3(ew_grid(total)), dim3(NT), 0, st, (const float*)x, ldx,
                       (const float*)gy, ldgy, N, H, W, C, (float*)gx, ldgx, accumulate);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_upsample_fwd(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, int scale, int mode,
                               void* y, int64_t ldy, void* stream) {
  DG_REQUIRE(x && y && N > 0 && H > 0 && W > 0 && C > 0 && scale >= 1 && mode >= 0 && mode <= 2);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  hipStream_t st = (hipStream_t)stream;
  return dtype == DG_BF16 ? up_fwd<bf16>(x, ldx, N, H, W, C, scale, mode, y, ldy, st)
                          : dtype == DG_F16 ? up_fwd<f16>(x, ldx, N, H, W, C, scale, mode, y, ldy, st) : up_fwd<float>(x, ldx, N, H, W, C, scale, mode, y, ldy, st);
}

extern "C" int dg_upsample_bwd(int dtype, const void* gy, int64_t ldgy, const void* gy2, int64_t ldgy2, int N, int H,
                               int W, int C, int scale, int mode, void* gx, int64_t ldgx, int accumulate,
                               void* stream) {
  DG_REQUIRE(gy && gx && N > 0 && H > 0 && W > 0 && C > 0 && scale >= 1 && mode >= 0 && mode <= 2);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  hipStream_t st = (hipStream_t)stream;
  return dtype == DG_BF16 ? up_bwd<bf16>(gy, ldgy, gy2, ldgy2, N, H, W, C, scale, mode, gx, ldgx, accumulate, st)
                          : dtype == DG_F16 ? up_bwd<f16>(gy, ldgy, gy2, ldgy2, N, H, W, C, scale, mode, gx, ldgx, accumulate, st) : up_bwd<float>(gy, ldgy, gy2, ldgy2, N, H, W, C, scale, mode, gx, ldgx, accumulate, st);
}


extern "C" int dg_maxpool_fwd(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, int k, int stride,
                              int pad, void* y, int64_t ldy, void* stream) {
  DG_REQUIRE(x && y && N > 0 && H > 0 && W > 0 && C > 0 && k > 0 && stride > 0 && pad >= 0 && 2 * pad <= k);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(C % V == 0 && ldx % V == 0 && ldy % V == 0);
  const int P = (H + 2 * pad - k) / stride + 1, Q = (W + 2 * pad - k) / stride + 1;
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)N * P * Q * (C / V);
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(maxpool_gen_fwd<bf16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const bf16*)x, ldx, N, H, W, C, k,
                       stride, pad, P, Q, (bf16*)y, ldy);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(maxpool_gen_fwd<f16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const f16*)x, ldx, N, H, W, C, k,
                       stride, pad, P, Q, (f16*)y, ldy);
  else
    hipLaunchKernelGGL(maxpool_gen_fwd<float>, dim3(ew_grid(total)), dim3(NT), 0, st, (const float*)x, ldx, N, H, W,
                       C, k, stride, pad, P, Q, (float*)y, ldy);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_maxpool_bwd(int dtype, const void* x, int64_t ldx, const void* gy, int64_t ldgy, int N, int H, int W,
                              int C, int k, int stride, int pad, void* gx, int64_t ldgx, int accumulate, void* stream) {
  DG_REQUIRE(x && gy && gx && N > 0 && H > 0 && W > 0 && C > 0 && k > 0 && stride > 0 && pad >= 0 && 2 * pad <= k);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(C % V == 0 && ldx % V == 0 && ldgy % V == 0 && ldgx % V == 0);
  const int P = (H + 2 * pad - k) / stride + 1, Q = (W + 2 * pad - k) / stride + 1;
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)N * H * W * (C / V);
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(maxpool_gen_bwd<bf16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const bf16*)x, ldx,
                       (const bf16*)gy, ldgy, N, H, W, C, k, stride, pad, P, Q, (bf16*)gx, ldgx, accumulate);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(maxpool_gen_bwd<f16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const f16*)x, ldx,
                       (const f16*)gy, ldgy, N, H, W, C, k, stride, pad, P, Q, (f16*)gx, ldgx, accumulate);
  else
    hipLaunchKernelGGL(maxpool_gen_bwd<float>, dim3(ew_grid(total)), dim3(NT), 0, st, (const float*)x, ldx,
                       (const float*)gy, ldgy, N, H, W, C, k, stride, pad, P, Q, (float*)gx, ldgx, accumulate);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_maxpool_fwd_idx(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, int k, int stride,
                                  int pad, void* y, int64_t ldy, unsigned char* idx, void* stream) {
  DG_REQUIRE(x && y && idx && N > 0 && H > 0 && W > 0 && C > 0 && k > 0 && k <= 15 && stride > 0 && pad >= 0 &&
             2 * pad <= k);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(C % V == 0 && ldx % V == 0 && ldy % V == 0 && (long long)N * H * W * (C / V) < (1LL << 30));
  const int P = (H + 2 * pad - k) / stride + 1, Q = (W + 2 * pad - k) / stride + 1;
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)N * P * Q * (C / V);
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(maxpool_idx_fwd<bf16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const bf16*)x, ldx, N, H, W, C, k,
                       stride, pad, P, Q, (bf16*)y, ldy, idx);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(maxpool_idx_fwd<f16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const f16*)x, ldx, N, H, W, C, k,
                       stride, pad, P, Q, (f16*)y, ldy, idx);
  else
    hipLaunchKernelGGL(maxpool_idx_fwd<float>, dim3(ew_grid(total)), dim3(NT), 0, st, (const float*)x, ldx, N, H, W,
                       C, k, stride, pad, P, Q, (float*)y, ldy, idx);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_maxpool_bwd_idx(int dtype, const unsigned char* idx, const void* gy, int64_t ldgy, int N, int H,
                                  int W, int C, int k, int stride, int pad, void* gx, int64_t ldgx, int accumulate,
                                  void* stream) {
  DG_REQUIRE(idx && gy && gx && N > 0 && H > 0 && W > 0 && C > 0 && k > 0 && k <= 15 && stride > 0 && pad >= 0 &&
             2 * pad <= k);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(C % V == 0 && ldgy % V == 0 && ldgx % V == 0 && (long long)N * H * W * (C / V) < (1LL << 30));
  const int P = (H + 2 * pad - k) / stride + 1, Q = (W + 2 * pad - k) / stride + 1;
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)N * H * W * (C / V);
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(maxpool_idx_bwd<bf16>, dim3(ew_grid(total)), dim3(NT), 0, st, idx, (const bf16*)gy, ldgy, N, H,
                       W, C, k, stride, pad, P, Q, (bf16*)gx, ldgx, accumulate);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(maxpool_idx_bwd<f16>, dim3(ew_grid(total)), dim3(NT), 0, st, idx, (const f16*)gy, ldgy, N, H,
                       W, C, k, stride, pad, P, Q, (f16*)gx, ldgx, accumulate);
  else
    hipLaunchKernelGGL(maxpool_idx_bwd<float>, dim3(ew_grid(total)), dim3(NT), 0, st, idx, (const float*)gy, ldgy, N,
                       H, W, C, k, stride, pad, P, Q, (float*)gx, ldgx, accumulate);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int64_t dg_cat_combine_part_rows(int N, int H, int W) {
  if (N <= 0 || H <= 0 || W <= 0) return DG_ERR_INVALID;
  return cat_nblk((long long)N * H * W);
}

extern "C" int dg_cat_combine(int dtype, const void* z1, int64_t ldz1, const void* z2, int64_t ldz2, const void* z3,
                              int64_t ldz3, int N, int H, int W, int C, const float* bias, void* z, int64_t ldz,
                              float* part, void* stream) {
  DG_REQUIRE(z1 && z2 && z3 && z && N > 0 && H > 0 && W > 0 && C > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(H % 4 == 0 && W % 4 == 0 && (long long)N * H * W < (1LL << 31) && C % V == 0 && 256 % (C / V) == 0 &&
               ldz1 % V == 0 && ldz2 % V == 0 &&
               ldz3 % V == 0 && ldz % V == 0);
  const long long M = (long long)N * H * W;
  const int nblk = cat_nblk(M);
  const long long ppb = (M + nblk - 1) / nblk;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(cat_combine_kernel<bf16>, dim3(nblk), dim3(NT), 0, st, (const bf16*)z1, (long long)ldz1,
                       (const bf16*)z2, (long long)ldz2, (const bf16*)z3, (long long)ldz3, H, W, M, C, ppb, bias,
                       (bf16*)z, (long long)ldz, part);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(cat_combine_kernel<f16>, dim3(nblk), dim3(NT), 0, st, (const f16*)z1, (long long)ldz1,
                       (const f16*)z2, (long long)ldz2, (const f16*)z3, (long long)ldz3, H, W, M, C, ppb, bias,
                       (f16*)z, (long long)ldz, part);
  else
    hipLaunchKernelGGL(cat_combine_kernel<float>, dim3(nblk), dim3(NT), 0, st, (const float*)z1, (long long)ldz1,
                       (const float*)z2, (long long)ldz2, (const float*)z3, (long long)ldz3, H, W, M, C, ppb, bias,
                       (float*)z, (long long)ldz, part);
  DG_CHECK_LAUNCH();
  return DG_OK;
}
