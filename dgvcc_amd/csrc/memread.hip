// Two-view consistency + memory read of DGModel_memadd / DGModel_final
// (models/models.py:116-125 forward_mem, :147-184 and :298-335 forward_train):
//   instance-norm statistics of y_den (F.instance_norm, eps 1e-5, biased var),
//   e_mask = |IN(y1) - IN(y2)| < err_thrs, masked + Dropout2d'd features,
//   row softmax over the 1024 memory slots for both views + JSD-MSE loss,
//   and the matching backward, plus the class-map combination of the cls head
//   (models/models.py:196-207, 323-327).
// The two GEMMs of the memory read run on the implicit-GEMM conv kernel (1x1).
#include "dg_common.h"
#include <algorithm>

namespace {

constexpr int NT = 256;

inline int ew_grid(long long n, int cap = 16384) {
  long long g = (n + NT - 1) / NT;
  return (int)std::max<long long>(1, std::min<long long>(g, cap));
}

// ------------------------------------------------------------ instance norm --
// grid (nb, N): block b of sample n reduces pixels [b*ppb, (b+1)*ppb) of that sample
template <typename T>
__global__ __launch_bounds__(NT) void in_stats_partial(const T* __restrict__ x, long long ldx, int HW, int C, int ppb,
                                                       float* __restrict__ part) {
  constexpr int V = 16 / (int)sizeof(T);
  __shared__ float sh[2][NT * V];
  const int n = blockIdx.y, nb = gridDim.x;
  const int tpp = C / V, rows = NT / tpp;
  const int tid = threadIdx.x, ch = tid % tpp, pl = tid / tpp;
  const T* xs = x + (long long)n * HW * ldx;
  float s1[V], s2[V], K[V];
#pragma unroll
  for (int e = 0; e < V; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  const int p0 = blockIdx.x * ppb, p1 = min(HW, p0 + ppb);
  if (pl < rows) {
    ldv(xs + ch * V, K);
    for (int p = p0 + pl; p < p1; p += rows) {
      float v[V];
      ldv(xs + (long long)p * ldx + ch * V, v);
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
    float* o = part + ((long long)n * nb + blockIdx.x) * 2 * C;
    o[c] = a; o[C + c] = b;
  }
}

template <typename T>
__global__ void in_stats_finalize(const T* __restrict__ x, long long ldx, int N, int HW, int C, int nb,
                                  const float* __restrict__ part, float eps, float* mean, float* invstd) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i % C;
  double a = 0.0, b = 0.0;
  for (int k = 0; k < nb; ++k) {
    const float* o = part + ((long long)n * nb + k) * 2 * C;
    a += o[c]; b += o[C + c];
  }
  const double K = (double)to_f(x[(long long)n * HW * ldx + c]);
  const double ms = a / HW;
  double var = b / HW - ms * ms;
  if (var < 0) var = 0;
  mean[i] = (float)(K + ms);
  invstd[i] = (float)(1.0 / sqrt(var + (double)eps));
}

// V consecutive per-(instance, channel) floats (16-B aligned: C % 4 == 0, c0 % V == 0); 1 when absent
template <int V>
__device__ __forceinline__ void ld_nc(const float* a, long long off, float (&o)[V]) {
  if (!a) {
#pragma unroll
    for (int e = 0; e < V; ++e) o[e] = 1.f;
    return;
  }
#pragma unroll
  for (int e = 0; e < V; e += 4) {
    const f4v t = *(const f4v*)(a + off + e);
    o[e] = t[0]; o[e + 1] = t[1]; o[e + 2] = t[2]; o[e + 3] = t[3];
  }
}

// The elementwise e_mask passes walk (pixel, V-channel chunk) items.  When the chunks of a pixel
// divide the block (NT % (C / V) == 0, e.g. the 512-channel x3) every thread keeps one chunk, so
// the item -> (pixel, channel) split is one division per block instead of two 64-bit divisions per
// item; the per-(instance, channel) statistics come in as 16-B loads and the V mask bytes as one
// store.
template <int V>
struct EwWalk {
  long long p, pstride, total;
  int c0, tpp;
  bool fixed;
  __device__ __forceinline__ EwWalk(long long M, int C) {
    tpp = C / V;
    total = M * tpp;
    fixed = NT % tpp == 0;
    const long long gt = blockIdx.x * (long long)NT + threadIdx.x;
    if (fixed) {
      c0 = (int)(threadIdx.x % tpp) * V;
      p = blockIdx.x * (long long)(NT / tpp) + threadIdx.x / tpp;
      pstride = (long long)gridDim.x * (NT / tpp);
    } else {
      p = gt;  // item index
      pstride = (long long)gridDim.x * NT;
      c0 = 0;
    }
  }
  __device__ __forceinline__ bool next(long long M, long long& px, int& ch) {
    if (fixed) {
      if (p >= M) return false;
      px = p;
      ch = c0;
    } else {
      if (p >= total) return false;
      px = p / tpp;
      ch = (int)(p % tpp) * V;
    }
    p += pstride;
    return true;
  }
};

template <int V>
__device__ __forceinline__ void st_mask(unsigned char* m, const unsigned char (&mk)[V]) {
  if constexpr (V == 8) {
    unsigned long long w = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) w |= (unsigned long long)mk[e] << (8 * e);
    *(unsigned long long*)m = w;
  } else {
    unsigned w = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) w |= (unsigned)mk[e] << (8 * e);
    *(unsigned*)m = w;
  }
}

// m_v = y_v * e * drop_v ; e = |(y1-mu1)*is1 - (y2-mu2)*is2| < thr  (stored as 0/1 bytes)
template <typename T>
__global__ __launch_bounds__(NT) void emask_fwd_kernel(const T* __restrict__ y1, const T* __restrict__ y2, long long ld,
                                                       int N, int HW, int C, const float* mu1, const float* is1,
                                                       const float* mu2, const float* is2, float thr,
                                                       const float* drop1, const float* drop2, T* __restrict__ m1,
                                                       T* __restrict__ m2, unsigned char* __restrict__ mask) {
  constexpr int V = 16 / (int)sizeof(T);
  const long long M = (long long)N * HW;
  EwWalk<V> w(M, C);
  long long p;
  int c0;
  while (w.next(M, p, c0)) {
    const long long nc = (M < (1ll << 31) ? (long long)((unsigned)p / (unsigned)HW) : p / HW) * C + c0;
    float a[V], b[V], ma[V], sa[V], mb[V], sb[V], da[V], db[V];
    ldv(y1 + p * ld + c0, a);
    ldv(y2 + p * ld + c0, b);
    ld_nc<V>(mu1, nc, ma);
    ld_nc<V>(is1, nc, sa);
    ld_nc<V>(mu2, nc, mb);
    ld_nc<V>(is2, nc, sb);
    ld_nc<V>(drop1, nc, da);
    ld_nc<V>(drop2, nc, db);
    unsigned char mk[V];
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const float ia = (a[e] - ma[e]) * sa[e];
      const float ib = (b[e] - mb[e]) * sb[e];
      const bool keep = fabsf(ia - ib) < thr;
      mk[e] = keep ? 1 : 0;
      a[e] = keep ? a[e] * da[e] : 0.f;
      b[e] = keep ? b[e] * db[e] : 0.f;
    }
    stv(m1 + p * C + c0, a);
    stv(m2 + p * C + c0, b);
    st_mask<V>(mask + p * C + c0, mk);
  }
}

// g_y_v = g_m_v * e * drop_v  (gy written with pixel stride ldgy; g_m dense)
template <typename T>
__global__ __launch_bounds__(NT) void emask_bwd_kernel(const T* __restrict__ gm1, const T* __restrict__ gm2, int N,
                                                       int HW, int C, const unsigned char* __restrict__ mask,
                                                       const float* drop1, const float* drop2, T* __restrict__ gy1,
                                                       T* __restrict__ gy2, long long ldgy) {
  constexpr int V = 16 / (int)sizeof(T);
  const long long M = (long long)N * HW;
  EwWalk<V> w(M, C);
  long long p;
  int c0;
  while (w.next(M, p, c0)) {
    const long long nc = (M < (1ll << 31) ? (long long)((unsigned)p / (unsigned)HW) : p / HW) * C + c0;
    float a[V], b[V], da[V], db[V];
    ldv(gm1 + p * C + c0, a);
    ldv(gm2 + p * C + c0, b);
    ld_nc<V>(drop1, nc, da);
    ld_nc<V>(drop2, nc, db);
    unsigned long long mw;
    if constexpr (V == 8) mw = *(const unsigned long long*)(mask + p * C + c0);
    else mw = *(const unsigned*)(mask + p * C + c0);
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const float k = ((mw >> (8 * e)) & 0xff) ? 1.f : 0.f;
      a[e] *= k * da[e];
      b[e] *= k * db[e];
    }
    stv(gy1 + p * ldgy + c0, a);
    stv(gy2 + p * ldgy + c0, b);
  }
}

// ------------------------------------------------------------ slot softmax ---
// One wave per pixel row of C (= 1024) logits; EPL elements per lane.
template <typename T>
__device__ __forceinline__ void load_row(const T* row, int lane, int C, float* v, int EPL) {
  constexpr int V = 16 / (int)sizeof(T);
  for (int j = 0; j < EPL; j += V) ldv(row + (long long)(j / V) * 64 * V + lane * V, v + j);
}
template <typename T>
__device__ __forceinline__ void store_row(T* row, int lane, float* v, int EPL) {
  constexpr int V = 16 / (int)sizeof(T);
  for (int j = 0; j < EPL; j += V) stv(row + (long long)(j / V) * 64 * V + lane * V, v + j);
}

template <typename T, int EPL>
__global__ __launch_bounds__(NT) void softmax_pair_fwd(const T* __restrict__ L1, const T* __restrict__ L2, int M, int C,
                                                       T* __restrict__ P1, T* __restrict__ P2,
                                                       float* __restrict__ part) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float acc = 0.f;
  for (long long r = (long long)blockIdx.x * 4 + w; r < M; r += (long long)gridDim.x * 4) {
    float a[EPL], b[EPL];
    load_row(L1 + r * C, lane, C, a, EPL);
    load_row(L2 + r * C, lane, C, b, EPL);
    float ma = -INFINITY, mb = -INFINITY;
#pragma unroll
    for (int j = 0; j < EPL; ++j) { ma = fmaxf(ma, a[j]); mb = fmaxf(mb, b[j]); }
    ma = wave_max(ma); mb = wave_max(mb);
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int j = 0; j < EPL; ++j) { a[j] = expf(a[j] - ma); sa += a[j]; b[j] = expf(b[j] - mb); sb += b[j]; }
    sa = wave_sum(sa); sb = wave_sum(sb);
    const float ra = 1.f / sa, rb = 1.f / sb;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      a[j] = to_f(from_f<T>(a[j] * ra));  // the loss sees the stored probabilities
      b[j] = to_f(from_f<T>(b[j] * rb));
      const float d = a[j] - b[j];
      acc = fmaf(d, d, acc);
    }
    store_row(P1 + r * C, lane, a, EPL);
    store_row(P2 + r * C, lane, b, EPL);
  }
  acc = wave_sum(acc);
  __shared__ float sh[4];
  if (lane == 0) sh[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

// one 64-thread block: lane-strided double sums, then a fixed xor tree (deterministic)
__global__ void sum_final(const float* __restrict__ part, int nblk, double denom, float* out) {
  double a = 0.0;
  for (int i = threadIdx.x; i < nblk; i += 64) a += part[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
  if (threadIdx.x == 0) out[0] = (float)(a / denom);
}

// gL_v = P_v * (gP_v' - sum(P_v * gP_v')),  gP1' = gP1 + k (P1 - P2), gP2' = gP2 - k (P1 - P2),
// k = 2 * coef[0] / (M*C)  (d/dP of mean((P1-P2)^2) times the upstream grad of loss_con)
template <typename T, int EPL>
__global__ __launch_bounds__(NT) void softmax_pair_bwd(const T* __restrict__ P1, const T* __restrict__ P2,
                                                       const T* __restrict__ G1, const T* __restrict__ G2, int M,
                                                       int C, const float* __restrict__ coef, T* __restrict__ GL1,
                                                       T* __restrict__ GL2) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float k = coef ? 2.f * coef[0] / ((float)M * (float)C) : 0.f;
  for (long long r = (long long)blockIdx.x * 4 + w; r < M; r += (long long)gridDim.x * 4) {
    float p1[EPL], p2[EPL], g1[EPL], g2[EPL];
    load_row(P1 + r * C, lane, C, p1, EPL);
    load_row(P2 + r * C, lane, C, p2, EPL);
    if (G1) load_row(G1 + r * C, lane, C, g1, EPL);
    else for (int j = 0; j < EPL; ++j) g1[j] = 0.f;
    if (G2) load_row(G2 + r * C, lane, C, g2, EPL);
    else for (int j = 0; j < EPL; ++j) g2[j] = 0.f;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      const float d = k * (p1[j] - p2[j]);
      g1[j] += d; g2[j] -= d;
      s1 = fmaf(p1[j], g1[j], s1);
      s2 = fmaf(p2[j], g2[j], s2);
    }
    s1 = wave_sum(s1); s2 = wave_sum(s2);
#pragma unroll
    for (int j = 0; j < EPL; ++j) { g1[j] = p1[j] * (g1[j] - s1); g2[j] = p2[j] * (g2[j] - s2); }
    store_row(GL1 + r * C, lane, g1, EPL);
    store_row(GL2 + r * C, lane, g2, EPL);
  }
}

// JSD of the two slot posteriors as models2.DensityRegressorM.forward_train computes it
// (models/models2.py:339-346): pm = (p1 + p2)/2,
//   loss_kl = 0.5/HW * (kl_div(log p1, pm, batchmean) + kl_div(log p2, pm, batchmean))
//           = sum_{rows, slots} pm (2 log pm - log p1 - log p2) / (2 M),  M = B*HW rows.
// log p is the log-softmax of the row (l - max - log sum); pm = 0 terms are 0 (xlogy).
template <typename T, int EPL>
__global__ __launch_bounds__(NT) void softmax_jsd_fwd(const T* __restrict__ L1, const T* __restrict__ L2, int M, int C,
                                                      T* __restrict__ P1, T* __restrict__ P2,
                                                      float* __restrict__ part) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float acc = 0.f;
  for (long long r = (long long)blockIdx.x * 4 + w; r < M; r += (long long)gridDim.x * 4) {
    float a[EPL], b[EPL], la[EPL], lb[EPL];
    load_row(L1 + r * C, lane, C, a, EPL);
    load_row(L2 + r * C, lane, C, b, EPL);
    float ma = -INFINITY, mb = -INFINITY;
#pragma unroll
    for (int j = 0; j < EPL; ++j) { ma = fmaxf(ma, a[j]); mb = fmaxf(mb, b[j]); }
    ma = wave_max(ma); mb = wave_max(mb);
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      la[j] = a[j] - ma; lb[j] = b[j] - mb;
      a[j] = expf(la[j]); sa += a[j]; b[j] = expf(lb[j]); sb += b[j];
    }
    sa = wave_sum(sa); sb = wave_sum(sb);
    const float ra = 1.f / sa, rb = 1.f / sb, dls = logf(sa) - logf(sb);
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      a[j] *= ra; b[j] *= rb;
      const float pm = 0.5f * (a[j] + b[j]);
      // 2 log pm - log p1 - log p2 = log1p((p1 - p2)^2 / (4 p1 p2)) = log1p(e^2 / (4 (1 + e))),
      // e = expm1(log p1 - log p2): no cancellation between the three O(log C) logs
      const float e = expm1f((la[j] - lb[j]) - dls);
      if (pm > 0.f) acc += pm * log1pf(e * e / (4.f * (1.f + e)));
    }
    store_row(P1 + r * C, lane, a, EPL);
    store_row(P2 + r * C, lane, b, EPL);
  }
  acc = wave_sum(acc);
  __shared__ float sh[4];
  if (lane == 0) sh[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

// d loss_kl / d l1_j = k (p1_j (A_j - S1 + 1) - pm_j),  A = log pm - (log p1 + log p2)/2,
// S1 = sum_j p1_j A_j, k = coef / (2 M); plus the readout's p1 (gP1 - <p1, gP1>).
template <typename T, int EPL>
__global__ __launch_bounds__(NT) void softmax_jsd_bwd(const T* __restrict__ P1, const T* __restrict__ P2,
                                                      const T* __restrict__ G1, const T* __restrict__ G2, int M,
                                                      int C, const float* __restrict__ coef, T* __restrict__ GL1,
                                                      T* __restrict__ GL2) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float k = coef ? coef[0] / (2.f * (float)M) : 0.f;
  for (long long r = (long long)blockIdx.x * 4 + w; r < M; r += (long long)gridDim.x * 4) {
    float p1[EPL], p2[EPL], g1[EPL], g2[EPL], A[EPL];
    load_row(P1 + r * C, lane, C, p1, EPL);
    load_row(P2 + r * C, lane, C, p2, EPL);
    if (G1) load_row(G1 + r * C, lane, C, g1, EPL);
    else for (int j = 0; j < EPL; ++j) g1[j] = 0.f;
    if (G2) load_row(G2 + r * C, lane, C, g2, EPL);
    else for (int j = 0; j < EPL; ++j) g2[j] = 0.f;
    float s1 = 0.f, s2 = 0.f, t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      const float pm = 0.5f * (p1[j] + p2[j]);
      // A = log pm - (log p1 + log p2)/2 = log1p((p1-p2)^2 / (4 p1 p2)) / 2 (cancellation-free)
      const float d = p1[j] - p2[j];
      A[j] = (p1[j] > 0.f && p2[j] > 0.f) ? 0.5f * log1pf(d * d / (4.f * p1[j] * p2[j]))
                                          : (pm > 0.f ? logf(pm) - 0.5f * (logf(p1[j]) + logf(p2[j])) : 0.f);
      s1 = fmaf(p1[j], g1[j], s1);
      s2 = fmaf(p2[j], g2[j], s2);
      t1 += p1[j] > 0.f ? p1[j] * A[j] : 0.f;
      t2 += p2[j] > 0.f ? p2[j] * A[j] : 0.f;
    }
    s1 = wave_sum(s1); s2 = wave_sum(s2); t1 = wave_sum(t1); t2 = wave_sum(t2);
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      const float pm = 0.5f * (p1[j] + p2[j]);
      const float a1 = p1[j] > 0.f ? p1[j] * (A[j] - t1 + 1.f) : 0.f;
      const float a2 = p2[j] > 0.f ? p2[j] * (A[j] - t2 + 1.f) : 0.f;
      g1[j] = p1[j] * (g1[j] - s1) + k * (a1 - pm);
      g2[j] = p2[j] * (g2[j] - s2) + k * (a2 - pm);
    }
    store_row(GL1 + r * C, lane, g1, EPL);
    store_row(GL2 + r * C, lane, g2, EPL);
  }
}

// loss_err = F.l1_loss(IN(y1), IN(y2)) (models/models2.py:334): block partial sums of
// |(y1-mu1)*is1 - (y2-mu2)*is2| over dense [N*HW][C] rows with pixel stride ld
template <typename T>
__global__ __launch_bounds__(NT) void in_l1_fwd_kernel(const T* __restrict__ y1, const T* __restrict__ y2,
                                                       long long ld, int N, int HW, int C, const float* mu1,
                                                       const float* is1, const float* mu2, const float* is2,
                                                       float* __restrict__ part) {
  constexpr int V = 16 / (int)sizeof(T);
  const int tpp = C / V;
  const long long total = (long long)N * HW * tpp;
  float acc = 0.f;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const long long p = i / tpp;
    const int c0 = (int)(i % tpp) * V;
    const int n = (int)(p / HW);
    float a[V], b[V];
    ldv(y1 + p * ld + c0, a);
    ldv(y2 + p * ld + c0, b);
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const int nc = n * C + c0 + e;
      acc += fabsf((a[e] - mu1[nc]) * is1[nc] - (b[e] - mu2[nc]) * is2[nc]);
    }
  }
  acc = wave_sum(acc);
  __shared__ float sh[NT / 64];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < NT / 64; ++k) t += sh[k];
    part[blockIdx.x] = t;
  }
}

// g_in1 = coef[0] * sgn(IN(y1) - IN(y2)) / (N*HW*C), g_in2 = -g_in1 (dense [N*HW][C])
template <typename T>
__global__ __launch_bounds__(NT) void in_l1_bwd_kernel(const T* __restrict__ y1, const T* __restrict__ y2,
                                                       long long ld, int N, int HW, int C, const float* mu1,
                                                       const float* is1, const float* mu2, const float* is2,
                                                       const float* __restrict__ coef, T* __restrict__ g1,
                                                       T* __restrict__ g2) {
  constexpr int V = 16 / (int)sizeof(T);
  const int tpp = C / V;
  const long long total = (long long)N * HW * tpp;
  const float k = coef[0] / ((float)N * (float)HW * (float)C);
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const long long p = i / tpp;
    const int c0 = (int)(i % tpp) * V;
    const int n = (int)(p / HW);
    float a[V], b[V];
    ldv(y1 + p * ld + c0, a);
    ldv(y2 + p * ld + c0, b);
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const int nc = n * C + c0 + e;
      const float d = (a[e] - mu1[nc]) * is1[nc] - (b[e] - mu2[nc]) * is2[nc];
      const float sg = d > 0.f ? k : (d < 0.f ? -k : 0.f);
      a[e] = sg;
      b[e] = -sg;
    }
    stv(g1 + p * C + c0, a);
    stv(g2 + p * C + c0, b);
  }
}

// single-view softmax (DGModel_mem.forward / memcls.forward)
template <typename T, int EPL>
__global__ __launch_bounds__(NT) void softmax_fwd(const T* __restrict__ L, int M, int C, T* __restrict__ P) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (long long r = (long long)blockIdx.x * 4 + w; r < M; r += (long long)gridDim.x * 4) {
    float a[EPL];
    load_row(L + r * C, lane, C, a, EPL);
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < EPL; ++j) m = fmaxf(m, a[j]);
    m = wave_max(m);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < EPL; ++j) { a[j] = expf(a[j] - m); s += a[j]; }
    s = wave_sum(s);
    const float rs = 1.f / s;
#pragma unroll
    for (int j = 0; j < EPL; ++j) a[j] *= rs;
    store_row(P + r * C, lane, a, EPL);
  }
}

template <typename T, int EPL>
__global__ __launch_bounds__(NT) void softmax_bwd(const T* __restrict__ P, const T* __restrict__ G, int M, int C,
                                                  T* __restrict__ GL) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (long long r = (long long)blockIdx.x * 4 + w; r < M; r += (long long)gridDim.x * 4) {
    float p[EPL], g[EPL];
    load_row(P + r * C, lane, C, p, EPL);
    load_row(G + r * C, lane, C, g, EPL);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < EPL; ++j) s = fmaf(p[j], g[j], s);
    s = wave_sum(s);
#pragma unroll
    for (int j = 0; j < EPL; ++j) g[j] = p[j] * (g[j] - s);
    store_row(GL + r * C, lane, g, EPL);
  }
}

// ------------------------------------------------------------ class maps -----
// c_v: [N][h][w] sigmoid outputs; cgt: [N][h][w] or NULL; outputs at (s*h, s*w):
// c_resized = clamp(up_nearest(cgt) + |up(c1>=thr) - up(c2>=thr)|, 0, 1), c_err.
// With c2 == NULL (single view): c_resized = cgt ? up(cgt) : up(c1>=thr).
__global__ void cls_combine_kernel(const float* __restrict__ c1, const float* __restrict__ c2,
                                   const float* __restrict__ cgt, int N, int h, int w, int s, float thr,
                                   float* __restrict__ cres, float* __restrict__ cerr) {
  const long long total = (long long)N * h * s * w * s;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int ow = (int)(i % (w * s));
    const long long t = i / (w * s);
    const int oh = (int)(t % (h * s));
    const int n = (int)(t / (h * s));
    const long long src = ((long long)n * h + oh / s) * w + ow / s;
    auto bin = [&](float v) { return v < thr ? 0.f : (v >= thr ? 1.f : v); };
    if (c2) {
      const float e = fabsf(bin(c1[src]) - bin(c2[src]));
      const float g = cgt ? cgt[src] : 0.f;
      cres[i] = fminf(fmaxf(g + e, 0.f), 1.f);
      if (cerr) cerr[i] = e;
    } else {
      cres[i] = cgt ? cgt[src] : bin(c1[src]);
    }
  }
}

__global__ void mul_kernel(const float* __restrict__ a, const float* __restrict__ b, long long n,
                           float* __restrict__ out) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = a[i] * b[i];
}

// ------------------------------------------------------- memory read + head --
// y_new = mem P (models/models.py:120-121) is consumed only by den_head, a 1x1 conv k -> 1 with
// bias and ReLU (models/models.py:112-114, 130-131, 328-329; models2.py DensityRegressorM), so
//   d = act(w . (mem P) + b) = act(v . P + b),   v = mem^T w   (one 1024-vector per step):
// the readout GEMM (2 k S FLOP per pixel) becomes a 1024-long dot fused into the softmax pass.
// Backward: g_ynew = gpre w^T is rank 1, hence
//   gP = gpre v (formed in registers, never stored),  dmem_readout = w u^T,  dw = mem u,  db = sum gpre,
//   u = sum_px gpre P  (per-block partial rows, reduced in a fixed order).
// NV = views per launch (1 or 2); LOSS: 0 none, 1 JSD-MSE mean((P1-P2)^2) (models.py:286-296),
// 2 KL-JSD of DensityRegressorM (models2.py:339-346).
__device__ __forceinline__ float mh_act(float s, int act) {
  if (act == 1) return s > 0.f ? s : 0.f;
  if (act == 2) return 1.f / (1.f + expf(-s));
  return s;
}
__device__ __forceinline__ float mh_gpre(float gy, float y, int act) {
  if (act == 1) return y > 0.f ? gy : 0.f;
  if (act == 2) return gy * y * (1.f - y);
  return gy;
}
// v at this lane's slots, in load_row's element order
template <typename T>
__device__ __forceinline__ void load_vec_as_row(const float* v, int lane, float* o, int EPL) {
  constexpr int V = 16 / (int)sizeof(T);
  for (int j = 0; j < EPL; ++j) o[j] = v[(j / V) * 64 * V + lane * V + (j % V)];
}

template <typename T, int EPL, int NV, int LOSS>
__global__ __launch_bounds__(NT) void softmax_head_fwd(const T* __restrict__ L1, const T* __restrict__ L2, int M,
                                                       int C, const float* __restrict__ v, const float* bias, int act,
                                                       T* __restrict__ P1, T* __restrict__ P2, float* __restrict__ yh1,
                                                       float* __restrict__ yh2, float* __restrict__ part) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float vv[EPL];
  load_vec_as_row<T>(v, lane, vv, EPL);
  const float hb = bias ? bias[0] : 0.f;
  float acc = 0.f;
  for (long long r = (long long)blockIdx.x * 4 + w; r < M; r += (long long)gridDim.x * 4) {
    float a[EPL], b[EPL], la[EPL], lb[EPL];
    load_row(L1 + r * C, lane, C, a, EPL);
    if (NV == 2) load_row(L2 + r * C, lane, C, b, EPL);
    float ma = -INFINITY, mb = -INFINITY;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      ma = fmaxf(ma, a[j]);
      if (NV == 2) mb = fmaxf(mb, b[j]);
    }
    ma = wave_max(ma);
    if (NV == 2) mb = wave_max(mb);
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      la[j] = a[j] - ma;
      a[j] = expf(la[j]);
      sa += a[j];
      if (NV == 2) { lb[j] = b[j] - mb; b[j] = expf(lb[j]); sb += b[j]; }
    }
    sa = wave_sum(sa);
    if (NV == 2) sb = wave_sum(sb);
    const float ra = 1.f / sa, rb = NV == 2 ? 1.f / sb : 0.f;
    const float dls = LOSS == 2 ? logf(sa) - logf(sb) : 0.f;
    float z1 = 0.f, z2 = 0.f;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      a[j] *= ra;
      if (NV == 2) b[j] *= rb;
      if (LOSS == 2) {  // cancellation-free 2 log pm - log p1 - log p2 (as softmax_jsd_fwd)
        const float pm = 0.5f * (a[j] + b[j]);
        const float e = expm1f((la[j] - lb[j]) - dls);
        if (pm > 0.f) acc += pm * log1pf(e * e / (4.f * (1.f + e)));
      }
      a[j] = to_f(from_f<T>(a[j]));  // the loss and the head see the stored probabilities
      if (NV == 2) b[j] = to_f(from_f<T>(b[j]));
      if (LOSS == 1) { const float d = a[j] - b[j]; acc = fmaf(d, d, acc); }
      z1 = fmaf(vv[j], a[j], z1);
      if (NV == 2) z2 = fmaf(vv[j], b[j], z2);
    }
    if (P1) store_row(P1 + r * C, lane, a, EPL);
    if (NV == 2 && P2) store_row(P2 + r * C, lane, b, EPL);
    z1 = wave_sum(z1);
    if (NV == 2) z2 = wave_sum(z2);
    if (lane == 0) {
      yh1[r] = mh_act(z1 + hb, act);
      if (NV == 2) yh2[r] = mh_act(z2 + hb, act);
    }
  }
  if (LOSS) {
    acc = wave_sum(acc);
    __shared__ float sh[4];
    if (lane == 0) sh[w] = acc;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
  }
}

// gL_v = P_v (gP_v - <P_v, gP_v>) with gP_v = gpre_v v + (loss term); u/db partials per block:
// part[blk][0:C] = sum_px sum_v gpre_v P_v, part[blk][C] = sum_px sum_v gpre_v.
// amax (may be NULL; zeroed by the launcher): CM = 0: [0] max |gL_1|, [1] max |gL_2|; CM = 1 (f32): per view
// v, at v * dg_amax_words(C), the operand maxima with channels of gL_v (word 0 the tensor's, 1 + s slot s's:
// the logits GEMMs' f16 x3 scales in the backward, per channel in their weight gradient), from per-lane
// running maxima of the lane's slots reduced over the block's waves in LDS.
template <typename T, int EPL, int NV, int LOSS, int CM = 0>
__global__ __launch_bounds__(NT) void softmax_head_bwd(const T* __restrict__ P1, const T* __restrict__ P2, int M,
                                                       int C, const float* __restrict__ v, int act,
                                                       const float* __restrict__ yh1, const float* __restrict__ yh2,
                                                       const float* __restrict__ gyh1, const float* __restrict__ gyh2,
                                                       const float* __restrict__ coef, T* __restrict__ GL1,
                                                       T* __restrict__ GL2, float* __restrict__ part,
                                                       float* __restrict__ amax) {
  constexpr int V = 16 / (int)sizeof(T);
  __shared__ float sh[4 * EPL * 64 + 4];
  float mx1 = 0.f, mx2 = 0.f;
  float cm1[CM ? EPL : 1], cm2[CM ? EPL : 1];  // CM: per-slot running maxima of |gL_v|
#pragma unroll
  for (int j = 0; j < (CM ? EPL : 1); ++j) { cm1[j] = 0.f; cm2[j] = 0.f; }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float vv[EPL], u[EPL];
  load_vec_as_row<T>(v, lane, vv, EPL);
#pragma unroll
  for (int j = 0; j < EPL; ++j) u[j] = 0.f;
  float sgb = 0.f;
  const float k = !coef ? 0.f : (LOSS == 1 ? 2.f * coef[0] / ((float)M * (float)C) : coef[0] / (2.f * (float)M));
  for (long long r = (long long)blockIdx.x * 4 + w; r < M; r += (long long)gridDim.x * 4) {
    const float q1 = gyh1 ? mh_gpre(gyh1[r], yh1[r], act) : 0.f;
    const float q2 = (NV == 2 && gyh2) ? mh_gpre(gyh2[r], yh2[r], act) : 0.f;
    sgb += q1 + q2;
    float p1[EPL], p2[EPL], g1[EPL], g2[EPL], A[EPL];
    load_row(P1 + r * C, lane, C, p1, EPL);
    if (NV == 2) load_row(P2 + r * C, lane, C, p2, EPL);
    float s1 = 0.f, s2 = 0.f, t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      u[j] = fmaf(q1, p1[j], u[j]);
      g1[j] = q1 * vv[j];
      if (NV == 2) {
        u[j] = fmaf(q2, p2[j], u[j]);
        g2[j] = q2 * vv[j];
      }
      if (LOSS == 1) {
        const float d = k * (p1[j] - p2[j]);
        g1[j] += d;
        g2[j] -= d;
      }
      if (LOSS == 2) {  // as softmax_jsd_bwd
        const float pm = 0.5f * (p1[j] + p2[j]);
        const float d = p1[j] - p2[j];
        A[j] = (p1[j] > 0.f && p2[j] > 0.f) ? 0.5f * log1pf(d * d / (4.f * p1[j] * p2[j]))
                                            : (pm > 0.f ? logf(pm) - 0.5f * (logf(p1[j]) + logf(p2[j])) : 0.f);
        t1 += p1[j] > 0.f ? p1[j] * A[j] : 0.f;
        t2 += p2[j] > 0.f ? p2[j] * A[j] : 0.f;
      }
      s1 = fmaf(p1[j], g1[j], s1);
      if (NV == 2) s2 = fmaf(p2[j], g2[j], s2);
    }
    s1 = wave_sum(s1);
    if (NV == 2) s2 = wave_sum(s2);
    if (LOSS == 2) { t1 = wave_sum(t1); t2 = wave_sum(t2); }
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      g1[j] = p1[j] * (g1[j] - s1);
      if (NV == 2) g2[j] = p2[j] * (g2[j] - s2);
      if (LOSS == 2) {
        const float pm = 0.5f * (p1[j] + p2[j]);
        const float a1 = p1[j] > 0.f ? p1[j] * (A[j] - t1 + 1.f) : 0.f;
        const float a2 = p2[j] > 0.f ? p2[j] * (A[j] - t2 + 1.f) : 0.f;
        g1[j] += k * (a1 - pm);
        g2[j] += k * (a2 - pm);
      }
    }
    if (GL1) store_row(GL1 + r * C, lane, g1, EPL);  // NULL: head gradients only (u, db)
    if (NV == 2 && GL2) store_row(GL2 + r * C, lane, g2, EPL);
#pragma unroll
    for (int j = 0; j < EPL; ++j) {
      if constexpr (CM) {
        cm1[j] = fmaxf(cm1[j], fabsf(g1[j]));
        if (NV == 2) cm2[j] = fmaxf(cm2[j], fabsf(g2[j]));
      } else {
        mx1 = fmaxf(mx1, fabsf(g1[j]));
        if (NV == 2) mx2 = fmaxf(mx2, fabsf(g2[j]));
      }
    }
  }
  // waves' u rows -> LDS at slot order, fixed-order sum over the 4 waves
#pragma unroll
  for (int j = 0; j < EPL; ++j) sh[w * EPL * 64 + (j / V) * 64 * V + lane * V + (j % V)] = u[j];
  if (lane == 0) sh[4 * EPL * 64 + w] = sgb;
  __syncthreads();
  float* o = part + (long long)blockIdx.x * (C + 1);
  for (int c = threadIdx.x; c < C; c += NT) o[c] = ((sh[c] + sh[C + c]) + sh[2 * C + c]) + sh[3 * C + c];
  if (threadIdx.x == 0) {
    const float* q = sh + 4 * EPL * 64;
    o[C] = ((q[0] + q[1]) + q[2]) + q[3];
  }
  if (amax) {  // uniform
    if constexpr (CM) {
      const int words = (int)dg_amax_words(C);
#pragma unroll
      for (int view = 0; view < NV; ++view) {
        __syncthreads();  // every thread is done reading sh (the u sums, or the previous view)
#pragma unroll
        for (int j = 0; j < EPL; ++j)
          sh[w * EPL * 64 + (j / V) * 64 * V + lane * V + (j % V)] = view == 0 ? cm1[j] : cm2[j];
        __syncthreads();
        float bm = 0.f;
        float* ov = amax + view * words;
        for (int c = threadIdx.x; c < C; c += NT) {
          const float m = fmaxf(fmaxf(sh[c], sh[C + c]), fmaxf(sh[2 * C + c], sh[3 * C + c]));
          bm = fmaxf(bm, m);
          if (m > 0.f) amax_fold((unsigned*)ov + 1 + c, m);
        }
        block_amax_commit(bm, ov);
      }
    } else {
      block_amax_commit(mx1, amax);
      if (NV == 2) {
        __syncthreads();  // block_amax_commit's LDS slots are reused
        block_amax_commit(mx2, amax + 1);
      }
    }
  }
}

// v[s] = sum_k w[k] mem[k][s]
__global__ void mem_head_vec_kernel(const float* __restrict__ mem, const float* __restrict__ w, int k, int S,
                                    float* __restrict__ v) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  float a = 0.f;
  for (int i = 0; i < k; ++i) a = fmaf(w[i], mem[(long long)i * S + s], a);
  v[s] = a;
}

// column sums of part[nblk][ncol] in double: grid (cdiv(ncol, 64), MH_CHUNKS); 4 row lanes per column
constexpr int MH_CHUNKS = 16;
__global__ __launch_bounds__(256) void mem_head_colsum(const float* __restrict__ part, int nblk, int ncol,
                                                       double* __restrict__ part2) {
  __shared__ double sh[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int per = (nblk + MH_CHUNKS - 1) / MH_CHUNKS;
  const int r0 = blockIdx.y * per, r1 = min(nblk, r0 + per);
  double a = 0.0;
  if (c < ncol)
    for (int r = r0 + rl; r < r1; r += 4) a += part[(long long)r * ncol + c];
  sh[rl][cl] = a;
  __syncthreads();
  if (rl == 0 && c < ncol) part2[(long long)blockIdx.y * ncol + c] = ((sh[0][cl] + sh[1][cl]) + sh[2][cl]) + sh[3][cl];
}

__global__ void mem_head_u(const double* __restrict__ part2, int ncol, float* __restrict__ u, float* gb) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncol) return;
  double a = 0.0;
  for (int i = 0; i < MH_CHUNKS; ++i) a += part2[(long long)i * ncol + c];
  u[c] = (float)a;
  if (c == ncol - 1 && gb) gb[0] = (float)a;
}

// block kk: dw[kk] = sum_s mem[kk][s] u[s] (fixed-order tree), dmem[kk][s] = w[kk] u[s]
__global__ __launch_bounds__(256) void mem_head_grads(const float* __restrict__ mem, const float* __restrict__ w,
                                                      const float* __restrict__ u, int S, float* __restrict__ dmem,
                                                      float* __restrict__ gw) {
  __shared__ float sh[256];
  const int kk = blockIdx.x;
  const float wk = w[kk];
  float a = 0.f;
  for (int s = threadIdx.x; s < S; s += 256) {
    const float us = u[s];
    a = fmaf(mem[(long long)kk * S + s], us, a);
    if (dmem) dmem[(long long)kk * S + s] = wk * us;
  }
  sh[threadIdx.x] = a;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) gw[kk] = sh[0];
}

#define SOFTMAX_DISPATCH(KERNEL, T, C, ...)                                                           \
  do {                                                                                                 \
    if ((C) == 1024) hipLaunchKernelGGL((KERNEL<T, 16>), dim3(grid), dim3(NT), 0, st, __VA_ARGS__);   \
    else if ((C) == 512) hipLaunchKernelGGL((KERNEL<T, 8>), dim3(grid), dim3(NT), 0, st, __VA_ARGS__); \
    else hipLaunchKernelGGL((KERNEL<T, 32>), dim3(grid), dim3(NT), 0, st, __VA_ARGS__);                \
  } while (0)

}  // namespace

extern "C" int64_t dg_instnorm_workspace(int N, int HW, int C) {
  if (N <= 0 || HW <= 0 || C <= 0) return DG_ERR_INVALID;
  const int nb = std::max(1, std::min(64, dg_cdiv(HW, 256)));
  return (int64_t)N * nb * 2 * C * 4;
}

extern "C" int dg_instnorm_stats(int dtype, const void* x, int64_t ldx, int N, int HW, int C, float eps, float* mean,
                                 float* invstd, void* workspace, void* stream) {
  DG_REQUIRE(x && mean && invstd && workspace && N > 0 && HW > 0 && C > 0);
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(C % V == 0 && C / V <= NT && ldx % V == 0);
  hipStream_t st = (hipStream_t)stream;
  const int nb = std::max(1, std::min(64, dg_cdiv(HW, 256)));
  const int ppb = dg_cdiv(HW, nb);
  if (dtype == DG_BF16) {
    hipLaunchKernelGGL(in_stats_partial<bf16>, dim3(nb, N), dim3(NT), 0, st, (const bf16*)x, ldx, HW, C, ppb,
                       (float*)workspace);
    DG_CHECK_LAUNCH();
    hipLaunchKernelGGL(in_stats_finalize<bf16>, dim3(dg_cdiv(N * C, 256)), dim3(256), 0, st, (const bf16*)x, ldx, N,
                       HW, C, nb, (const float*)workspace, eps, mean, invstd);
  } else if (dtype == DG_F16) {
    hipLaunchKernelGGL(in_stats_partial<f16>, dim3(nb, N), dim3(NT), 0, st, (const f16*)x, ldx, HW, C, ppb,
                       (float*)workspace);
    DG_CHECK_LAUNCH();
    hipLaunchKernelGGL(in_stats_finalize<f16>, dim3(dg_cdiv(N * C, 256)), dim3(256), 0, st, (const f16*)x, ldx, N,
                       HW, C, nb, (const float*)workspace, eps, mean, invstd);
  } else {
    hipLaunchKernelGGL(in_stats_partial<float>, dim3(nb, N), dim3(NT), 0, st, (const float*)x, ldx, HW, C, ppb,
                       (float*)workspace);
    DG_CHECK_LAUNCH();
    hipLaunchKernelGGL(in_stats_finalize<float>, dim3(dg_cdiv(N * C, 256)), dim3(256), 0, st, (const float*)x, ldx,
                       N, HW, C, nb, (const float*)workspace, eps, mean, invstd);
  }
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_emask_fwd(int dtype, const void* y1, const void* y2, int64_t ld, int N, int HW, int C,
                            const float* mu1, const float* is1, const float* mu2, const float* is2, float thr,
                            const float* drop1, const float* drop2, void* m1, void* m2, unsigned char* mask,
                            void* stream) {
  DG_REQUIRE(y1 && y2 && mu1 && is1 && mu2 && is2 && m1 && m2 && mask && N > 0 && HW > 0 && C > 0);
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(C % V == 0 && ld % V == 0);
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)N * HW * (C / V);
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(emask_fwd_kernel<bf16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const bf16*)y1,
                       (const bf16*)y2, ld, N, HW, C, mu1, is1, mu2, is2, thr, drop1, drop2, (bf16*)m1, (bf16*)m2,
                       mask);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(emask_fwd_kernel<f16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const f16*)y1,
                       (const f16*)y2, ld, N, HW, C, mu1, is1, mu2, is2, thr, drop1, drop2, (f16*)m1, (f16*)m2,
                       mask);
  else
    hipLaunchKernelGGL(emask_fwd_kernel<float>, dim3(ew_grid(total)), dim3(NT), 0, st, (const float*)y1,
                       (const float*)y2, ld, N, HW, C, mu1, is1, mu2, is2, thr, drop1, drop2, (float*)m1, (float*)m2,
                       mask);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_emask_bwd(int dtype, const void* gm1, const void* gm2, int N, int HW, int C,
                            const unsigned char* mask, const float* drop1, const float* drop2, void* gy1, void* gy2,
                            int64_t ldgy, void* stream) {
  DG_REQUIRE(gm1 && gm2 && mask && gy1 && gy2 && N > 0 && HW > 0 && C > 0);
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(C % V == 0 && ldgy % V == 0);
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)N * HW * (C / V);
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(emask_bwd_kernel<bf16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const bf16*)gm1,
                       (const bf16*)gm2, N, HW, C, mask, drop1, drop2, (bf16*)gy1, (bf16*)gy2, ldgy);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(emask_bwd_kernel<f16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const f16*)gm1,
                       (const f16*)gm2, N, HW, C, mask, drop1, drop2, (f16*)gy1, (f16*)gy2, ldgy);
  else
    hipLaunchKernelGGL(emask_bwd_kernel<float>, dim3(ew_grid(total)), dim3(NT), 0, st, (const float*)gm1,
                       (const float*)gm2, N, HW, C, mask, drop1, drop2, (float*)gy1, (float*)gy2, ldgy);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int64_t dg_softmax_workspace(int M) {
  if (M <= 0) return DG_ERR_INVALID;
  return (int64_t)std::min(4096, dg_cdiv(M, 4)) * 4;
}

#define SOFTMAX_C_OK(C) ((C) == 1024 || (C) == 512 || (C) == 2048)

extern "C" int dg_softmax_pair_fwd(int dtype, const void* L1, const void* L2, int M, int C, void* P1, void* P2,
                                   float* loss_con, void* workspace, void* stream) {
  DG_REQUIRE(L1 && L2 && P1 && P2 && loss_con && workspace && M > 0);
  DG_SUPPORTED(SOFTMAX_C_OK(C));
  hipStream_t st = (hipStream_t)stream;
  const int grid = std::min(4096, dg_cdiv(M, 4));
  if (dtype == DG_BF16)
    SOFTMAX_DISPATCH(softmax_pair_fwd, bf16, C, (const bf16*)L1, (const bf16*)L2, M, C, (bf16*)P1, (bf16*)P2,
                     (float*)workspace);
  else if (dtype == DG_F16)
    SOFTMAX_DISPATCH(softmax_pair_fwd, f16, C, (const f16*)L1, (const f16*)L2, M, C, (f16*)P1, (f16*)P2,
                     (float*)workspace);
  else
    SOFTMAX_DISPATCH(softmax_pair_fwd, float, C, (const float*)L1, (const float*)L2, M, C, (float*)P1, (float*)P2,
                     (float*)workspace);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(sum_final, dim3(1), dim3(64), 0, st, (const float*)workspace, grid, (double)M * C, loss_con);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_softmax_pair_bwd(int dtype, const void* P1, const void* P2, const void* G1, const void* G2, int M,
                                   int C, const float* coef, void* GL1, void* GL2, void* stream) {
  DG_REQUIRE(P1 && P2 && GL1 && GL2 && M > 0);
  DG_SUPPORTED(SOFTMAX_C_OK(C));
  hipStream_t st = (hipStream_t)stream;
  const int grid = std::min(4096, dg_cdiv(M, 4));
  if (dtype == DG_BF16)
    SOFTMAX_DISPATCH(softmax_pair_bwd, bf16, C, (const bf16*)P1, (const bf16*)P2, (const bf16*)G1, (const bf16*)G2,
                     M, C, coef, (bf16*)GL1, (bf16*)GL2);
  else if (dtype == DG_F16)
    SOFTMAX_DISPATCH(softmax_pair_bwd, f16, C, (const f16*)P1, (const f16*)P2, (const f16*)G1, (const f16*)G2,
                     M, C, coef, (f16*)GL1, (f16*)GL2);
  else
    SOFTMAX_DISPATCH(softmax_pair_bwd, float, C, (const float*)P1, (const float*)P2, (const float*)G1,
                     (const float*)G2, M, C, coef, (float*)GL1, (float*)GL2);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_softmax_jsd_fwd(int dtype, const void* L1, const void* L2, int M, int C, void* P1, void* P2,
                                  float* loss_kl, void* workspace, void* stream) {
  DG_REQUIRE(L1 && L2 && P1 && P2 && loss_kl && workspace && M > 0);
  DG_SUPPORTED(SOFTMAX_C_OK(C));
  hipStream_t st = (hipStream_t)stream;
  const int grid = std::min(4096, dg_cdiv(M, 4));
  if (dtype == DG_BF16)
    SOFTMAX_DISPATCH(softmax_jsd_fwd, bf16, C, (const bf16*)L1, (const bf16*)L2, M, C, (bf16*)P1, (bf16*)P2,
                     (float*)workspace);
  else if (dtype == DG_F16)
    SOFTMAX_DISPATCH(softmax_jsd_fwd, f16, C, (const f16*)L1, (const f16*)L2, M, C, (f16*)P1, (f16*)P2,
                     (float*)workspace);
  else
    SOFTMAX_DISPATCH(softmax_jsd_fwd, float, C, (const float*)L1, (const float*)L2, M, C, (float*)P1, (float*)P2,
                     (float*)workspace);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(sum_final, dim3(1), dim3(64), 0, st, (const float*)workspace, grid, 2.0 * (double)M, loss_kl);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_softmax_jsd_bwd(int dtype, const void* P1, const void* P2, const void* G1, const void* G2, int M,
                                  int C, const float* coef, void* GL1, void* GL2, void* stream) {
  DG_REQUIRE(P1 && P2 && GL1 && GL2 && M > 0);
  DG_SUPPORTED(SOFTMAX_C_OK(C));
  hipStream_t st = (hipStream_t)stream;
  const int grid = std::min(4096, dg_cdiv(M, 4));
  if (dtype == DG_BF16)
    SOFTMAX_DISPATCH(softmax_jsd_bwd, bf16, C, (const bf16*)P1, (const bf16*)P2, (const bf16*)G1, (const bf16*)G2,
                     M, C, coef, (bf16*)GL1, (bf16*)GL2);
  else if (dtype == DG_F16)
    SOFTMAX_DISPATCH(softmax_jsd_bwd, f16, C, (const f16*)P1, (const f16*)P2, (const f16*)G1, (const f16*)G2,
                     M, C, coef, (f16*)GL1, (f16*)GL2);
  else
    SOFTMAX_DISPATCH(softmax_jsd_bwd, float, C, (const float*)P1, (const float*)P2, (const float*)G1,
                     (const float*)G2, M, C, coef, (float*)GL1, (float*)GL2);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int64_t dg_in_l1_workspace(int N, int HW, int C) {
  if (N <= 0 || HW <= 0 || C <= 0) return DG_ERR_INVALID;
  return (int64_t)ew_grid((long long)N * HW * C / 4, 4096) * 4;
}

extern "C" int dg_in_l1_fwd(int dtype, const void* y1, const void* y2, int64_t ld, int N, int HW, int C,
                            const float* mu1, const float* is1, const float* mu2, const float* is2, float* loss,
                            void* workspace, void* stream) {
  DG_REQUIRE(y1 && y2 && mu1 && is1 && mu2 && is2 && loss && workspace && N > 0 && HW > 0 && C > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(C % V == 0 && ld % V == 0);
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)N * HW * (C / V);
  const int grid = ew_grid(total, 4096);
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(in_l1_fwd_kernel<bf16>, dim3(grid), dim3(NT), 0, st, (const bf16*)y1, (const bf16*)y2, ld, N,
                       HW, C, mu1, is1, mu2, is2, (float*)workspace);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(in_l1_fwd_kernel<f16>, dim3(grid), dim3(NT), 0, st, (const f16*)y1, (const f16*)y2, ld, N,
                       HW, C, mu1, is1, mu2, is2, (float*)workspace);
  else
    hipLaunchKernelGGL(in_l1_fwd_kernel<float>, dim3(grid), dim3(NT), 0, st, (const float*)y1, (const float*)y2, ld,
                       N, HW, C, mu1, is1, mu2, is2, (float*)workspace);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(sum_final, dim3(1), dim3(64), 0, st, (const float*)workspace, grid, (double)N * HW * C, loss);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_in_l1_bwd(int dtype, const void* y1, const void* y2, int64_t ld, int N, int HW, int C,
                            const float* mu1, const float* is1, const float* mu2, const float* is2, const float* coef,
                            void* g1, void* g2, void* stream) {
  DG_REQUIRE(y1 && y2 && mu1 && is1 && mu2 && is2 && coef && g1 && g2 && N > 0 && HW > 0 && C > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(C % V == 0 && ld % V == 0);
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)N * HW * (C / V);
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(in_l1_bwd_kernel<bf16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const bf16*)y1,
                       (const bf16*)y2, ld, N, HW, C, mu1, is1, mu2, is2, coef, (bf16*)g1, (bf16*)g2);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(in_l1_bwd_kernel<f16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const f16*)y1,
                       (const f16*)y2, ld, N, HW, C, mu1, is1, mu2, is2, coef, (f16*)g1, (f16*)g2);
  else
    hipLaunchKernelGGL(in_l1_bwd_kernel<float>, dim3(ew_grid(total)), dim3(NT), 0, st, (const float*)y1,
                       (const float*)y2, ld, N, HW, C, mu1, is1, mu2, is2, coef, (float*)g1, (float*)g2);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_softmax_fwd(int dtype, const void* L, int M, int C, void* P, void* stream) {
  DG_REQUIRE(L && P && M > 0);
  DG_SUPPORTED(SOFTMAX_C_OK(C));
  hipStream_t st = (hipStream_t)stream;
  const int grid = std::min(4096, dg_cdiv(M, 4));
  if (dtype == DG_BF16) SOFTMAX_DISPATCH(softmax_fwd, bf16, C, (const bf16*)L, M, C, (bf16*)P);
  else if (dtype == DG_F16) SOFTMAX_DISPATCH(softmax_fwd, f16, C, (const f16*)L, M, C, (f16*)P);
  else SOFTMAX_DISPATCH(softmax_fwd, float, C, (const float*)L, M, C, (float*)P);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_softmax_bwd(int dtype, const void* P, const void* G, int M, int C, void* GL, void* stream) {
  DG_REQUIRE(P && G && GL && M > 0);
  DG_SUPPORTED(SOFTMAX_C_OK(C));
  hipStream_t st = (hipStream_t)stream;
  const int grid = std::min(4096, dg_cdiv(M, 4));
  if (dtype == DG_BF16) SOFTMAX_DISPATCH(softmax_bwd, bf16, C, (const bf16*)P, (const bf16*)G, M, C, (bf16*)GL);
  else if (dtype == DG_F16) SOFTMAX_DISPATCH(softmax_bwd, f16, C, (const f16*)P, (const f16*)G, M, C, (f16*)GL);
  else SOFTMAX_DISPATCH(softmax_bwd, float, C, (const float*)P, (const float*)G, M, C, (float*)GL);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_cls_combine(const float* c1, const float* c2, const float* cgt, int N, int h, int w, int scale,
                              float thr, float* c_resized, float* c_err, void* stream) {
  DG_REQUIRE(c1 && c_resized && N > 0 && h > 0 && w > 0 && scale >= 1);
  const long long total = (long long)N * h * w * scale * scale;
  hipLaunchKernelGGL(cls_combine_kernel, dim3(ew_grid(total)), dim3(NT), 0, (hipStream_t)stream, c1, c2, cgt, N, h,
                     w, scale, thr, c_resized, c_err);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_mul_f32(const float* a, const float* b, int64_t n, float* out, void* stream) {
  DG_REQUIRE(a && b && out && n > 0);
  hipLaunchKernelGGL(mul_kernel, dim3(ew_grid(n)), dim3(NT), 0, (hipStream_t)stream, a, b, (long long)n, out);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// ------------------------------------------------------- memory read + head --
namespace {

inline int mh_grid(int M) { return std::min(4096, dg_cdiv(M, 4)); }

struct MhLayout {  // workspace: part f32 [grid][C+1] | part2 f64 [MH_CHUNKS][C+1] | u f32 [C+1]
  int grid;
  size_t part, part2, u, total;
  MhLayout(int M, int C) {
    grid = mh_grid(M);
    part = 0;
    part2 = ((size_t)grid * (C + 1) * 4 + 255) / 256 * 256;
    u = part2 + ((size_t)MH_CHUNKS * (C + 1) * 8 + 255) / 256 * 256;
    total = u + (size_t)(C + 1) * 4;
  }
};

template <typename T, int NV, int LOSS>
void mh_fwd_c(int C, int grid, hipStream_t st, const void* L1, const void* L2, int M, const float* v,
              const float* bias, int act, void* P1, void* P2, float* yh1, float* yh2, float* part) {
#define MHF(E) hipLaunchKernelGGL((softmax_head_fwd<T, E, NV, LOSS>), dim3(grid), dim3(NT), 0, st, (const T*)L1, \
                                  (const T*)L2, M, C, v, bias, act, (T*)P1, (T*)P2, yh1, yh2, part)
  if (C == 1024) MHF(16);
  else if (C == 512) MHF(8);
  else MHF(32);
#undef MHF
}

template <typename T, int NV, int LOSS>
void mh_bwd_c(int C, int grid, hipStream_t st, const void* P1, const void* P2, int M, const float* v, int act,
              const float* yh1, const float* yh2, const float* g1, const float* g2, const float* coef, void* GL1,
              void* GL2, float* part, float* amax) {
#define MHB(E, CM_)                                                                                                \
  hipLaunchKernelGGL((softmax_head_bwd<T, E, NV, LOSS, CM_>), dim3(grid), dim3(NT), 0, st, (const T*)P1, (const T*)P2, \
                     M, C, v, act, yh1, yh2, g1, g2, coef, (T*)GL1, (T*)GL2, part, amax)
  if constexpr (std::is_same<T, float>::value) {  // f32 logit gradients: per-slot operand maxima
    if (amax) {
      if (C == 1024) MHB(16, 1);
      else if (C == 512) MHB(8, 1);
      else MHB(32, 1);
      return;
    }
  }
  if (C == 1024) MHB(16, 0);
  else if (C == 512) MHB(8, 0);
  else MHB(32, 0);
#undef MHB
}

template <typename T>
void mh_fwd_t(int nv, int loss, int C, int grid, hipStream_t st, const void* L1, const void* L2, int M,
              const float* v, const float* bias, int act, void* P1, void* P2, float* yh1, float* yh2, float* part) {
  if (nv == 1) mh_fwd_c<T, 1, 0>(C, grid, st, L1, L2, M, v, bias, act, P1, P2, yh1, yh2, part);
  else if (loss == 0) mh_fwd_c<T, 2, 0>(C, grid, st, L1, L2, M, v, bias, act, P1, P2, yh1, yh2, part);
  else if (loss == 1) mh_fwd_c<T, 2, 1>(C, grid, st, L1, L2, M, v, bias, act, P1, P2, yh1, yh2, part);
  else mh_fwd_c<T, 2, 2>(C, grid, st, L1, L2, M, v, bias, act, P1, P2, yh1, yh2, part);
}

template <typename T>
void mh_bwd_t(int nv, int loss, int C, int grid, hipStream_t st, const void* P1, const void* P2, int M,
              const float* v, int act, const float* yh1, const float* yh2, const float* g1, const float* g2,
              const float* coef, void* GL1, void* GL2, float* part, float* amax) {
  if (nv == 1) mh_bwd_c<T, 1, 0>(C, grid, st, P1, P2, M, v, act, yh1, yh2, g1, g2, coef, GL1, GL2, part, amax);
  else if (loss == 0) mh_bwd_c<T, 2, 0>(C, grid, st, P1, P2, M, v, act, yh1, yh2, g1, g2, coef, GL1, GL2, part, amax);
  else if (loss == 1) mh_bwd_c<T, 2, 1>(C, grid, st, P1, P2, M, v, act, yh1, yh2, g1, g2, coef, GL1, GL2, part, amax);
  else mh_bwd_c<T, 2, 2>(C, grid, st, P1, P2, M, v, act, yh1, yh2, g1, g2, coef, GL1, GL2, part, amax);
}

}  // namespace

extern "C" int64_t dg_mem_head_workspace(int M, int C) {
  if (M <= 0 || !SOFTMAX_C_OK(C)) return DG_ERR_INVALID;
  return (int64_t)MhLayout(M, C).total;
}

extern "C" int dg_mem_head_vec(const float* mem, const float* w, int k, int S, float* v, void* stream) {
  DG_REQUIRE(mem && w && v && k > 0 && S > 0);
  hipLaunchKernelGGL(mem_head_vec_kernel, dim3(dg_cdiv(S, 256)), dim3(256), 0, (hipStream_t)stream, mem, w, k, S, v);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_softmax_head_fwd(int dtype, int nviews, int loss, const void* L1, const void* L2, int M, int C,
                                   const float* v, const float* bias, int act, void* P1, void* P2, float* yh1,
                                   float* yh2, float* loss_out, void* workspace, void* stream) {
  DG_REQUIRE(L1 && v && yh1 && M > 0 && (nviews == 1 || nviews == 2) && loss >= 0 && loss <= 2 && act >= 0 &&
             act <= 2);
  DG_REQUIRE(nviews == 1 ? loss == 0 : (L2 && yh2));
  DG_REQUIRE(!loss || (loss_out && workspace));
  DG_SUPPORTED(SOFTMAX_C_OK(C));
  hipStream_t st = (hipStream_t)stream;
  const int grid = mh_grid(M);
  float* part = (float*)workspace;
  if (dtype == DG_BF16) mh_fwd_t<bf16>(nviews, loss, C, grid, st, L1, L2, M, v, bias, act, P1, P2, yh1, yh2, part);
  else if (dtype == DG_F16) mh_fwd_t<f16>(nviews, loss, C, grid, st, L1, L2, M, v, bias, act, P1, P2, yh1, yh2, part);
  else if (dtype == DG_F32) mh_fwd_t<float>(nviews, loss, C, grid, st, L1, L2, M, v, bias, act, P1, P2, yh1, yh2, part);
  else return DG_ERR_INVALID;
  DG_CHECK_LAUNCH();
  if (loss) {
    const double denom = loss == 1 ? (double)M * C : 2.0 * (double)M;
    hipLaunchKernelGGL(sum_final, dim3(1), dim3(64), 0, st, (const float*)workspace, grid, denom, loss_out);
    DG_CHECK_LAUNCH();
  }
  return DG_OK;
}

extern "C" int dg_softmax_head_bwd(int dtype, int nviews, int loss, const void* P1, const void* P2, int M, int C,
                                   const float* v, int act, const float* yh1, const float* yh2, const float* gyh1,
                                   const float* gyh2, const float* coef, void* GL1, void* GL2, void* workspace,
                                   float* amax, void* stream) {
  DG_REQUIRE(P1 && v && yh1 && workspace && M > 0 && (nviews == 1 || nviews == 2) && loss >= 0 && loss <= 2);
  DG_REQUIRE(nviews == 1 ? loss == 0 : (P2 && yh2));
  DG_REQUIRE(nviews == 1 || !GL1 == !GL2);  // logit gradients for every view or none
  DG_SUPPORTED(SOFTMAX_C_OK(C));
  hipStream_t st = (hipStream_t)stream;
  const int grid = mh_grid(M);
  float* part = (float*)workspace;
  // amax: f32, nviews x dg_amax_words(C) floats (per-slot maxima per view); 16-bit, one word per view
  const size_t am_bytes = dtype == DG_F32 ? (size_t)nviews * dg_amax_words(C) * 4 : 8;
  if (amax && hipMemsetAsync(amax, 0, am_bytes, st) != hipSuccess) return DG_ERR_HIP;
  if (dtype == DG_BF16)
    mh_bwd_t<bf16>(nviews, loss, C, grid, st, P1, P2, M, v, act, yh1, yh2, gyh1, gyh2, coef, GL1, GL2, part, amax);
  else if (dtype == DG_F16)
    mh_bwd_t<f16>(nviews, loss, C, grid, st, P1, P2, M, v, act, yh1, yh2, gyh1, gyh2, coef, GL1, GL2, part, amax);
  else if (dtype == DG_F32)
    mh_bwd_t<float>(nviews, loss, C, grid, st, P1, P2, M, v, act, yh1, yh2, gyh1, gyh2, coef, GL1, GL2, part, amax);
  else return DG_ERR_INVALID;
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_mem_head_grads(void* workspace, int M, int C, const float* mem, const float* w, int k,
                                 float* dmem, float* gw, float* gb, void* stream) {
  DG_REQUIRE(workspace && mem && w && gw && M > 0 && k > 0);
  DG_SUPPORTED(SOFTMAX_C_OK(C));
  hipStream_t st = (hipStream_t)stream;
  const MhLayout lay(M, C);
  char* base = (char*)workspace;
  const int ncol = C + 1;
  hipLaunchKernelGGL(mem_head_colsum, dim3(dg_cdiv(ncol, 64), MH_CHUNKS), dim3(256), 0, st,
                     (const float*)(base + lay.part), lay.grid, ncol, (double*)(base + lay.part2));
  DG_CHECK_LAUNCH();
  float* u = (float*)(base + lay.u);
  hipLaunchKernelGGL(mem_head_u, dim3(dg_cdiv(ncol, 256)), dim3(256), 0, st, (const double*)(base + lay.part2), ncol,
                     u, gb);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(mem_head_grads, dim3(k), dim3(256), 0, st, mem, w, (const float*)u, C, dmem, gw);
  DG_CHECK_LAUNCH();
  return DG_OK;
}
