// Whitening kernels of the domain-generalisation trunks.
//
// ISW (models/ISW/instance_whitening.py:19-39, models/ISW/__init__.py:93-120):
//   the per-instance Gram matrices f_cor = w w^T/(HW-1) + eps I are produced by
//   dg_conv2d_wgrad (a 1x1 "weight gradient" of w against itself, one launch per
//   instance); here live the masked-L1 loss + its gradient and the
//   variance-of-covariance statistic of cal_covstat.
//
// SW (models/SW/ops/switchwhiten.py:84-183), sw_type 2 (BW + IW), groups of 16
// channels: statistics with f32 MFMA (16x16x4: one group's 16x16 covariance per
// wave), Newton-Schulz whitening matrices in one 256-thread block per group
// (thread = matrix element), and a fused whiten+affine+ReLU apply.  Backward is
// the exact adjoint (Newton iterations recomputed in LDS, no autograd tape).
#include "dg_common.h"
#include <algorithm>
#include <cstdlib>

extern "C" int64_t dg_instnorm_workspace(int N, int HW, int C);
extern "C" int dg_instnorm_stats(int dtype, const void* x, int64_t ldx, int N, int HW, int C, float eps, float* mean,
                                 float* invstd, void* workspace, void* stream);

namespace {

// ============================================================== ISW ========
// grid (chunks, B): partial sums of |f_ij| * mask_ij
__global__ __launch_bounds__(256) void iw_loss_partial(const float* __restrict__ fraw, int C, float inv_hw1, float eps,
                                                       const float* __restrict__ mask, float* __restrict__ part) {
  const int b = blockIdx.y;
  const long long CC = (long long)C * C;
  const float* f = fraw + b * CC;
  float s = 0.f;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < CC; e += (long long)gridDim.x * 256) {
    const int i = (int)(e / C), j = (int)(e % C);
    const float v = fmaf(f[e], inv_hw1, i == j ? eps : 0.f);
    s = fmaf(fabsf(v), mask[e], s);
  }
  __shared__ float sh[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[b * gridDim.x + blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

// loss (+)= out_scale * sum_b max(0, sum_e / ns) / B
__global__ void iw_loss_finalize(const float* __restrict__ part, int B, int nch, const float* __restrict__ ns,
                                 float out_scale, int accumulate, float* __restrict__ loss) {
  if (threadIdx.x != 0) return;
  double tot = 0.0;
  for (int b = 0; b < B; ++b) {
    double s = 0.0;
    for (int k = 0; k < nch; ++k) s += part[b * nch + k];
    s /= (double)ns[0];
    tot += s > 0.0 ? s : 0.0;
  }
  const float v = (float)(tot / B) * out_scale;
  loss[0] = accumulate ? loss[0] + v : v;
}

// gsym[b] = k * (M∘sgn(f) + (M∘sgn(f))^T),  k = coef*out_scale*inv_hw1/(ns*B)
// (the clamp(min=0) of instance_whitening_loss is inactive: its argument is a sum
// of absolute values with margin 0, models/ISW/cov_settings.py:47)
__global__ __launch_bounds__(256) void iw_loss_grad(const float* __restrict__ fraw, int B, int C, float inv_hw1,
                                                    float eps, const float* __restrict__ mask,
                                                    const float* __restrict__ ns, const float* __restrict__ coef,
                                                    float out_scale, float* __restrict__ gsym) {
  const long long CC = (long long)C * C, total = CC * B;
  const float k = (coef ? coef[0] : 1.f) * out_scale * inv_hw1 / (ns[0] * (float)B);
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long b = e / CC, r = e % CC;
    const int i = (int)(r / C), j = (int)(r % C);
    const float* f = fraw + b * CC;
    const float vij = fmaf(f[r], inv_hw1, i == j ? eps : 0.f);
    const float vji = fmaf(f[(long long)j * C + i], inv_hw1, i == j ? eps : 0.f);
    const float sij = vij > 0.f ? 1.f : (vij < 0.f ? -1.f : 0.f);
    const float sji = vji > 0.f ? 1.f : (vji < 0.f ? -1.f : 0.f);
    gsym[e] = k * (mask[r] * sij + mask[(long long)j * C + i] * sji);
  }
}

// var over instances (unbiased) of f_ij * [j > i]  (cal_covstat, __init__.py:96-103)
__global__ __launch_bounds__(256) void iw_cov_var(const float* __restrict__ fraw, int B, int C, float inv_hw1,
                                                  float* __restrict__ var, int accumulate) {
  const long long CC = (long long)C * C;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < CC; e += (long long)gridDim.x * 256) {
    const int i = (int)(e / C), j = (int)(e % C);
    float v = 0.f;
    if (j > i) {
      double m = 0.0;
      for (int b = 0; b < B; ++b) m += (double)(fraw[b * CC + e] * inv_hw1);
      m /= B;
      double s = 0.0;
      for (int b = 0; b < B; ++b) {
        const double d = (double)(fraw[b * CC + e] * inv_hw1) - m;
        s += d * d;
      }
      v = (float)(s / (B - 1));  // B == 1 -> NaN, as torch.var
    }
    var[e] = accumulate ? var[e] + v : v;
  }
}

// ============================================================== SW =========
constexpr int SWC = 16;  // channels per whitening group (sw_cfg num_pergroup)
constexpr int SW_MAXT = 8;

// Per-(n, block) partial 16x16 covariance of every group, centred on the
// instance mean: part[n][blk][g][16*16].  The block stages PT pixels x C channels in LDS
// as centred f32 (16-B vector loads of whole pixel rows: coalesced), then a wave owns groups
// w, w+4, ...; one f32 MFMA 16x16x4 consumes 4 pixels x 16 channels with a == b (lane l reads
// xc[p + l/16][g*16 + l%16]), so D = sum_p xc xc^T.  Rows are padded by 16 floats so the
// four pixel rows of one MFMA operand fall in distinct LDS banks.
__host__ __device__ inline int sw_pt(int C) { return C <= 128 ? 32 : 16; }

template <typename T>
__device__ __forceinline__ void sw_stage(const T* __restrict__ src, long long ld, int pb, int p1, int C, int PT,
                                         const float* __restrict__ sub, float* __restrict__ dst, int RS) {
  constexpr int V = 16 / (int)sizeof(T);
  const int cpr = C / V;
  for (int e = threadIdx.x; e < PT * cpr; e += 256) {
    const int r = e / cpr, cc = (e - r * cpr) * V;
    const int p = pb + r;
    float v[V];
    if (p < p1) {
      ldv(src + (long long)p * ld + cc, v);
      if (sub) {
#pragma unroll
        for (int k = 0; k < V; ++k) v[k] -= sub[cc + k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < V; ++k) v[k] = 0.f;
    }
#pragma unroll
    for (int k = 0; k < V; k += 4) *(f4v*)(dst + r * RS + cc + k) = f4v{v[k], v[k + 1], v[k + 2], v[k + 3]};
  }
}

template <typename T, int MAXG>
__global__ __launch_bounds__(256) void sw_cov_partial(const T* __restrict__ x, long long ldx, int HW, int C, int ppb,
                                                      const float* __restrict__ mu, float* __restrict__ part) {
  extern __shared__ float sm[];  // Xs[PT][C + 16] | mu[C]
  const int n = blockIdx.y, nb = gridDim.x, G = C / SWC, RS = C + 16, PT = sw_pt(C);
  float* Xs = sm;
  float* ms = sm + PT * RS;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kq = lane >> 4, ch = lane & 15;
  for (int e = threadIdx.x; e < C; e += 256) ms[e] = mu[(long long)n * C + e];
  f4v acc[MAXG];
#pragma unroll
  for (int q = 0; q < MAXG; ++q) acc[q] = f4v{0.f, 0.f, 0.f, 0.f};
  const int p0 = blockIdx.x * ppb, p1 = min(HW, p0 + ppb);
  const T* xn = x + (long long)n * HW * ldx;
  for (int pb = p0; pb < p1; pb += PT) {
    __syncthreads();
    sw_stage(xn, ldx, pb, p1, C, PT, ms, Xs, RS);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < MAXG; ++q) {
      const int g = wave + 4 * q;
      if (g < G) {
        for (int k = 0; k < PT; k += 4) {
          const float v = Xs[(k + kq) * RS + g * SWC + ch];
          acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(v, v, acc[q], 0, 0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < MAXG; ++q) {
    const int g = wave + 4 * q;
    if (g < G) {
      float* o = part + (((long long)n * nb + blockIdx.x) * G + g) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[(kq * 4 + r) * 16 + ch] = acc[q][r];
    }
  }
}

// 16x16 product for thread t = (i, j):  sum_k A(i,k) B(k,j), optional transposes.
template <bool TA, bool TB>
__device__ __forceinline__ float mm16(const float* A, const float* B, int i, int j) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const float a = TA ? A[k * 16 + i] : A[i * 16 + k];
    const float b = TB ? B[j * 16 + k] : B[k * 16 + j];
    s = fmaf(a, b, s);
  }
  return s;
}

__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const float r = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return r;
}

__device__ __forceinline__ void softmax2(const float* w, float& a0, float& a1) {
  const float m = fmaxf(w[0], w[1]);
  const float e0 = expf(w[0] - m), e1 = expf(w[1] - m);
  a0 = e0 / (e0 + e1);
  a1 = e1 / (e0 + e1);
}

// Newton-Schulz whitening matrix of S (LDS, 256): P_{k+1} = 1.5 P_k - 0.5 P_k^3 (S/tr S),
// W = P_T sqrt(1/tr S).  Ps[k] (k = 0..T) kept in LDS when Ps != nullptr.
struct SwLds {
  float S[256], A[256], P[256], P2[256], P3[256], X[256], Y[256], G[256];
  float red[4];
  float vec[4][16];
};

__device__ float sw_newton(SwLds& L, float* Ps, int T, int t) {
  const int i = t >> 4, j = t & 15;
  // trace
  __shared__ float tr_s;
  if (t == 0) {
    float tr = 0.f;
    for (int d = 0; d < 16; ++d) tr += L.S[d * 17];
    tr_s = tr;
  }
  __syncthreads();
  const float r = 1.f / tr_s;
  L.A[t] = L.S[t] * r;
  L.P[t] = i == j ? 1.f : 0.f;
  if (Ps) Ps[t] = L.P[t];
  __syncthreads();
  for (int k = 0; k < T; ++k) {
    const float p2 = mm16<false, false>(L.P, L.P, i, j);
    L.P2[t] = p2;
    __syncthreads();
    const float p3 = mm16<false, false>(L.P2, L.P, i, j);
    L.P3[t] = p3;
    __syncthreads();
    const float q = mm16<false, false>(L.P3, L.A, i, j);
    const float pn = 1.5f * L.P[t] - 0.5f * q;
    __syncthreads();
    L.P[t] = pn;
    if (Ps) Ps[(k + 1) * 256 + t] = pn;
    __syncthreads();
  }
  return r;
}

// Save layout (floats): mu_in[N][C] | cov_in[N][G][256] | mu_bn[C] | cov_bn[G][256]
//                       | aff[N][G][256] | bias[N][C]
// Batch moments (doubles, per group): S1[16] = sum_n mu_n, S2[256] = sum_n (cov_n + mu_n mu_n^T).
// They are the only cross-instance quantities of BW, so SyncSwitchWhiten reduces exactly
// these [G][272] doubles over ranks between sw_inst_stats and sw_finalize.
constexpr int SW_MOM = 272;

// One block per (group, instance): the instance covariance (partials / HW).
__global__ __launch_bounds__(256) void sw_inst_stats(const float* __restrict__ part, int N, int nb, int HW, int C,
                                                     float* __restrict__ save) {
  const int g = blockIdx.x, n = blockIdx.y, G = C / SWC, t = threadIdx.x;
  float* cov_in = save + (long long)N * C;
  double s = 0.0;
  const float* pp = part + ((long long)n * nb * G + g) * 256 + t;
  const long long ks = (long long)G * 256;
  int k = 0;
  for (; k + 8 <= nb; k += 8) {  // 8 loads in flight, added in block order (same sum)
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = pp[(k + u) * ks];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; k < nb; ++k) s += pp[k * ks];
  cov_in[((long long)n * G + g) * 256 + t] = (float)(s / HW);
}

// One block per group: the batch moments over this rank's instances, in instance order.
__global__ __launch_bounds__(256) void sw_moments(int N, int C, const float* __restrict__ save,
                                                  double* __restrict__ moments) {
  const int g = blockIdx.x, G = C / SWC, t = threadIdx.x, i = t >> 4, j = t & 15;
  const float* mu_in = save;
  const float* cov_in = save + (long long)N * C;
  double s2 = 0.0, s1 = 0.0;
  for (int n = 0; n < N; ++n) {
    const float ci = cov_in[((long long)n * G + g) * 256 + t];
    const double mi = mu_in[(long long)n * C + g * 16 + i], mj = mu_in[(long long)n * C + g * 16 + j];
    s2 += (double)ci + mi * mj;
    if (t < 16) s1 += mu_in[(long long)n * C + g * 16 + t];
  }
  moments[(long long)g * SW_MOM + 16 + t] = s2;
  if (t < 16) moments[(long long)g * SW_MOM + t] = s1;
}

// One block per (group, instance): batch mean/cov from the (possibly all-reduced) moments
// over `count` instances (or the running statistics in eval; recomputed per block, the
// instance-0 block writes them and updates the running statistics), then this instance's
// Newton-Schulz whitening matrix folded with the affine.
__global__ __launch_bounds__(256) void sw_finalize(const double* __restrict__ moments, double count, int N, int C,
                                                   int T, float eps, float momentum, const float* mean_w,
                                                   const float* var_w, const float* gamma, const float* beta,
                                                   float* running_mean, float* running_cov, int training,
                                                   float* __restrict__ save) {
  __shared__ SwLds L;
  const int g = blockIdx.x, n = blockIdx.y, G = C / SWC, t = threadIdx.x, i = t >> 4, j = t & 15;
  const bool lead = n == 0;
  float* mu_in = save;
  float* cov_in = mu_in + (long long)N * C;
  float* mu_bn = cov_in + (long long)N * G * 256;
  float* cov_bn = mu_bn + C;
  float* aff = cov_bn + (long long)G * 256;
  float* bias = aff + (long long)N * G * 256;
  __shared__ double mbd[16];
  if (t < 16) mbd[t] = moments[(long long)g * SW_MOM + t] / count;
  __syncthreads();
  float cbn;
  if (training) {
    cbn = (float)(moments[(long long)g * SW_MOM + 16 + t] / count - mbd[i] * mbd[j]);
    if (t < 16) {
      const float mb = (float)mbd[t];
      L.vec[0][t] = mb;
      if (lead) {
        mu_bn[g * 16 + t] = mb;
        float* rm = running_mean + g * 16 + t;
        *rm = *rm * momentum + (1.f - momentum) * mb;
      }
    }
    if (lead) {
      cov_bn[g * 256 + t] = cbn;
      float* rc = running_cov + g * 256 + t;
      *rc = *rc * momentum + (1.f - momentum) * cbn;
    }
  } else {
    if (t < 16) {
      const float mb = running_mean[g * 16 + t];
      L.vec[0][t] = mb;
      if (lead) mu_bn[g * 16 + t] = mb;
    }
    cbn = running_cov[g * 256 + t];
    if (lead) cov_bn[g * 256 + t] = cbn;
  }
  __syncthreads();
  float a0, a1, b0, b1;
  softmax2(mean_w, a0, a1);
  softmax2(var_w, b0, b1);
  const float ci = cov_in[((long long)n * G + g) * 256 + t];
  L.S[t] = b0 * cbn + b1 * ci + (i == j ? eps : 0.f);
  if (t < 16) L.vec[1][t] = a0 * L.vec[0][t] + a1 * mu_in[(long long)n * C + g * 16 + t];  // mixed mean
  __syncthreads();
  const float r = sw_newton(L, nullptr, T, t);
  const float w = L.P[t] * sqrtf(r);
  const float gi = gamma ? gamma[g * 16 + i] : 1.f;
  L.X[t] = gi * w;
  __syncthreads();
  aff[((long long)n * G + g) * 256 + t] = L.X[t];
  if (t < 16) {
    float sacc = 0.f;
    for (int k = 0; k < 16; ++k) sacc = fmaf(L.X[t * 16 + k], L.vec[1][k], sacc);
    bias[(long long)n * C + g * 16 + t] = (beta ? beta[g * 16 + t] : 0.f) - sacc;
  }
}

// y[p][g*16+i] = act(sum_j aff[n][g][i][j] x[p][g*16+j] + bias[n][g*16+i]);  thread = (pixel, group)
template <typename T>
__global__ __launch_bounds__(256) void sw_apply(const T* __restrict__ x, long long ldx, int HW, int C, int ppb,
                                                const float* __restrict__ aff, const float* __restrict__ bias, int act,
                                                T* __restrict__ y, long long ldy) {
  extern __shared__ float sm[];  // [G][273]
  const int n = blockIdx.y, G = C / SWC;
  for (int e = threadIdx.x; e < G * 256; e += 256) sm[(e >> 8) * 273 + (e & 255)] = aff[(long long)n * G * 256 + e];
  for (int e = threadIdx.x; e < C; e += 256) sm[(e >> 4) * 273 + 256 + (e & 15)] = bias[(long long)n * C + e];
  __syncthreads();
  const int g = threadIdx.x % G, pl = threadIdx.x / G, rows = 256 / G;
  if (pl >= rows) return;
  const float* A = sm + g * 273;
  const int p0 = blockIdx.x * ppb, p1 = min(HW, p0 + ppb);
  for (int p = p0 + pl; p < p1; p += rows) {
    const long long pp = (long long)n * HW + p;
    float v[16], o[16];
    constexpr int V = 16 / (int)sizeof(T);
#pragma unroll
    for (int q = 0; q < 16; q += V) ldv(x + pp * ldx + g * 16 + q, v + q);
#pragma unroll
    for (int a = 0; a < 16; ++a) {
      float s = A[256 + a];
#pragma unroll
      for (int b = 0; b < 16; ++b) s = fmaf(A[a * 16 + b], v[b], s);
      o[a] = (act == 1 && s < 0.f) ? 0.f : s;
    }
#pragma unroll
    for (int q = 0; q < 16; q += V) stv(y + pp * ldy + g * 16 + q, o + q);
  }
}

// ---------------------------------------------------------------- SW bwd --
// Per-(n, block) partials: GXc[g] = sum_p ge_p (x_p - mu_n)^T (MFMA, a = ge, b = xc)
// and sgy[g] = sum_p ge_p, where ge = gy * (y > 0) when act == 1.  ge and xc are staged
// PT pixels at a time in LDS as f32 (coalesced 16-B loads), as in sw_cov_partial.
// part layout: [n][blk][g][256 + 16]
template <typename T, int MAXG>
__global__ __launch_bounds__(256) void sw_bwd_partial(const T* __restrict__ gy, long long ldg, const T* __restrict__ y,
                                                      long long ldy, const T* __restrict__ x, long long ldx, int HW,
                                                      int C, int ppb, int act, const float* __restrict__ mu,
                                                      float* __restrict__ part) {
  extern __shared__ float sm[];  // Gs[PT][C + 16] | Xs[PT][C + 16] | mu[C]
  const int n = blockIdx.y, nb = gridDim.x, G = C / SWC, RS = C + 16, PT = sw_pt(C);
  float* Gs = sm;
  float* Xs = sm + PT * RS;
  float* ms = Xs + PT * RS;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kq = lane >> 4, ch = lane & 15;
  for (int e = threadIdx.x; e < C; e += 256) ms[e] = mu[(long long)n * C + e];
  f4v acc[MAXG];
  float sg[MAXG];
#pragma unroll
  for (int q = 0; q < MAXG; ++q) {
    acc[q] = f4v{0.f, 0.f, 0.f, 0.f};
    sg[q] = 0.f;
  }
  const int p0 = blockIdx.x * ppb, p1 = min(HW, p0 + ppb);
  const long long base = (long long)n * HW;
  constexpr int V = 16 / (int)sizeof(T);
  const int cpr = C / V;
  for (int pb = p0; pb < p1; pb += PT) {
    __syncthreads();
    sw_stage(x + base * ldx, ldx, pb, p1, C, PT, ms, Xs, RS);
    for (int e = threadIdx.x; e < PT * cpr; e += 256) {
      const int r = e / cpr, cc = (e - r * cpr) * V;
      const long long p = pb + r;
      float v[V];
      if (p < p1) {
        ldv(gy + (base + p) * ldg + cc, v);
        if (act == 1) {
          float yv[V];
          ldv(y + (base + p) * ldy + cc, yv);
#pragma unroll
          for (int k = 0; k < V; ++k) v[k] = yv[k] > 0.f ? v[k] : 0.f;
        }
      } else {
#pragma unroll
        for (int k = 0; k < V; ++k) v[k] = 0.f;
      }
#pragma unroll
      for (int k = 0; k < V; k += 4) *(f4v*)(Gs + r * RS + cc + k) = f4v{v[k], v[k + 1], v[k + 2], v[k + 3]};
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < MAXG; ++q) {
      const int g = wave + 4 * q;
      if (g < G) {
        for (int k = 0; k < PT; k += 4) {
          const int o = (k + kq) * RS + g * SWC + ch;
          const float ge = Gs[o];
          sg[q] += ge;
          acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(ge, Xs[o], acc[q], 0, 0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < MAXG; ++q) {
    const int g = wave + 4 * q;
    float s = sg[q];
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    if (g < G) {
      float* o = part + (((long long)n * nb + blockIdx.x) * G + g) * 272;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[(kq * 4 + r) * 16 + ch] = acc[q][r];
      if (kq == 0) o[256 + ch] = s;
    }
  }
}

// One block per (group, instance): exact adjoint of sw_finalize for that instance (phase A).
// coef layout: [n][g][ K(256) | L(256) | c(16) ]  so that
//   dx_p = K ge_p + L (x_p - mu_n) + c.
// The cross-instance sums leave as per-(n, g) rows of npart [n][g][SW_NP]:
//   dcov_bn(256) | dmu_bn(16) | dgamma(16) | dbeta(16) | da0-da1 db0-db1
// and sw_bwd_reduce adds them in instance order.
constexpr int SW_NP = 320;
__global__ __launch_bounds__(256) void sw_bwd_small(const float* __restrict__ part, int N, int nb, int HW, int C, int T,
                                                    float eps, const float* mean_w, const float* var_w,
                                                    const float* gamma, const float* __restrict__ save,
                                                    float* __restrict__ coef, float* __restrict__ npart) {
  __shared__ SwLds L;
  __shared__ float Ps[(SW_MAXT + 1) * 256];
  __shared__ float mv[4][16];  // mu_bn, mixed mean, mu_n, sgy
  const int g = blockIdx.x, n = blockIdx.y, G = C / SWC, t = threadIdx.x, i = t >> 4, j = t & 15;
  const float* mu_in = save;
  const float* cov_in = mu_in + (long long)N * C;
  const float* mu_bn = cov_in + (long long)N * G * 256;
  const float* cov_bn = mu_bn + C;
  float a0, a1, b0, b1;
  softmax2(mean_w, a0, a1);
  softmax2(var_w, b0, b1);
  const float cbn = cov_bn[g * 256 + t];
  const float gam_i = gamma ? gamma[g * 16 + i] : 1.f;
  const float gam_j = gamma ? gamma[g * 16 + j] : 1.f;
  const float ci = cov_in[((long long)n * G + g) * 256 + t];
  // reduce partials of this (n, g)
  float gx = 0.f, sg = 0.f;
  {
    const float* o0 = part + ((long long)n * nb * G + g) * 272;
    const long long ks = (long long)G * 272;
    const int ts = t < 16 ? 256 + t : t;  // lanes >= 16: a harmless re-read, not added
    int k = 0;
    for (; k + 8 <= nb; k += 8) {  // 8 blocks' loads in flight, added in block order (same sums)
      float v[8], w[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[u] = o0[(k + u) * ks + t];
        w[u] = o0[(k + u) * ks + ts];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        gx += v[u];
        if (t < 16) sg += w[u];
      }
    }
    for (; k < nb; ++k) {
      gx += o0[k * ks + t];
      if (t < 16) sg += o0[k * ks + 256 + t];
    }
  }
  if (t < 16) {
    mv[0][t] = mu_bn[g * 16 + t];
    mv[2][t] = mu_in[(long long)n * C + g * 16 + t];
    mv[1][t] = a0 * mv[0][t] + a1 * mv[2][t];
    mv[3][t] = sg;
  }
  L.S[t] = b0 * cbn + b1 * ci + (i == j ? eps : 0.f);
  __syncthreads();
  const float r = sw_newton(L, Ps, T, t);
  const float sr = sqrtf(r);
  const float PT = L.P[t];
  const float W = PT * sr;
  // H = GXc - sgy (m - mu_n)^T ; dW = diag(gamma) H
  const float H = gx - mv[3][i] * (mv[1][j] - mv[2][j]);
  const float dW = gam_i * H;
  // dgamma_i = sum_j W_ij H_ij ; dbeta_i = sgy_i
  float wh = W * H;
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) wh += __shfl_xor(wh, o, 16);
  float* np = npart + ((long long)n * G + g) * SW_NP;
  if (j == 0) {
    np[272 + i] = wh;
    np[288 + i] = mv[3][i];
  }
  // K = W^T diag(gamma): K_ij = W_ji gamma_j  (store W into X for the transpose)
  L.X[t] = W;
  __syncthreads();
  float* cf = coef + ((long long)n * G + g) * 528;
  cf[t] = L.X[j * 16 + i] * gam_j;
  // dm_t = -sum_k W_kt gamma_k sgy_k  (t < 16)
  float dm = 0.f;
  if (t < 16) {
    for (int k = 0; k < 16; ++k) dm -= L.X[k * 16 + t] * (gamma ? gamma[g * 16 + k] : 1.f) * mv[3][k];
  }
  // Newton adjoint: G = dP_T
  L.G[t] = dW * sr;
  const float dr_w = block_sum256(dW * PT, L.red) * 0.5f / sr;
  float dA = 0.f;
  __syncthreads();
  for (int k = T - 1; k >= 0; --k) {
    const float* P = Ps + k * 256;
    L.P2[t] = mm16<false, false>(P, P, i, j);           // P^2
    L.X[t] = mm16<false, false>(P, L.A, i, j);          // P A
    __syncthreads();
    L.P3[t] = mm16<false, false>(L.P2, P, i, j);        // P^3
    L.Y[t] = mm16<false, false>(L.P2, L.A, i, j);       // P^2 A
    __syncthreads();
    dA -= 0.5f * mm16<true, false>(L.P3, L.G, i, j);    // (P^3)^T G
    const float t1 = mm16<false, true>(L.G, L.Y, i, j);  // G (P^2 A)^T
    const float u = mm16<false, true>(L.G, L.X, i, j);   // G (P A)^T
    const float v = mm16<false, true>(L.G, L.A, i, j);   // G A^T
    __syncthreads();
    L.Y[t] = u;
    L.X[t] = v;
    __syncthreads();
    const float t2 = mm16<true, false>(P, L.Y, i, j);      // P^T G (P A)^T
    const float t3 = mm16<true, false>(L.P2, L.X, i, j);   // (P^2)^T G A^T
    const float gn = 1.5f * L.G[t] - 0.5f * (t1 + t2 + t3);
    __syncthreads();
    L.G[t] = gn;
    __syncthreads();
  }
  // A = S r ; r = 1/tr(S)
  const float dr = dr_w + block_sum256(dA * L.S[t], L.red);
  const float dS = r * dA + (i == j ? -r * r * dr : 0.f);
  // mixing-weight adjoints in difference form: softmax2's backward only needs da0 - da1
  // (dtheta = a0 a1 (da0 - da1) (1, -1)), and summing dm (mu_bn - mu_n), dS (C_bn - C_n)
  // directly avoids the cancellation of two large sums
  const float ddb = block_sum256(dS * (cbn - ci), L.red);
  np[t] = b0 * dS;  // this instance's dcov_bn
  // D_n = b1 (dS + dS^T) / HW  (stored in the L slot; E added by sw_bwd_coef)
  L.X[t] = dS;
  __syncthreads();
  cf[256 + t] = b1 * (dS + L.X[j * 16 + i]) / (float)HW;
  if (t < 16) {
    np[256 + t] = a0 * dm;               // dmu_bn
    cf[512 + t] = a1 * dm / (float)HW;  // dmu_n / HW (completed by sw_bwd_coef)
  }
  const float dda = block_sum256(t < 16 ? dm * (mv[0][t] - mv[2][t]) : 0.f, L.red);
  if (t == 0) {
    np[304] = dda;
    np[305] = ddb;
  }
}

// One block per group: the batch-statistics adjoints (bmoments, all-reduced over ranks by
// SyncSwitchWhiten), dgamma/dbeta and the mixing-weight partials, summed over this rank's
// instances in order.
__global__ __launch_bounds__(256) void sw_bwd_reduce(const float* __restrict__ npart, int N, int C,
                                                     double* __restrict__ bmoments, float* dgamma, float* dbeta,
                                                     float* __restrict__ wpart) {
  const int g = blockIdx.x, G = C / SWC, t = threadIdx.x;
  double dc = 0.0, dmu = 0.0, dga = 0.0, dbe = 0.0, w4 = 0.0;
  for (int n = 0; n < N; ++n) {
    const float* np = npart + ((long long)n * G + g) * SW_NP;
    dc += np[t];
    if (t < 16) {
      dmu += np[256 + t];
      dga += np[272 + t];
      dbe += np[288 + t];
    } else if (t < 18) {
      w4 += np[304 + t - 16];
    }
  }
  bmoments[(long long)g * SW_MOM + 16 + t] = dc;
  if (t < 16) {
    bmoments[(long long)g * SW_MOM + t] = dmu;
    if (dgamma) dgamma[g * 16 + t] = (float)dga;
    if (dbeta) dbeta[g * 16 + t] = (float)dbe;
  } else if (t < 18) {
    wpart[g * 4 + t - 16] = (float)w4;
  }
}

// Completes coef with the batch terms: Esym = (dC + dC^T)/(count HW) added to L,
// c += Esym (mu_n - mu_bn) + dmu_bn/(count HW); count = images over all ranks.
__global__ __launch_bounds__(256) void sw_bwd_coef(const double* __restrict__ bmoments, double count, int N, int HW,
                                                   int C, const float* __restrict__ save, float* __restrict__ coef) {
  __shared__ float E[256];
  __shared__ float mb[16], dmu[16];
  const int g = blockIdx.x, G = C / SWC, t = threadIdx.x, i = t >> 4, j = t & 15;
  const float* mu_in = save;
  const float* mu_bn = mu_in + (long long)N * C + (long long)N * G * 256;
  const double* bm = bmoments + (long long)g * SW_MOM;
  const double den = count * (double)HW;
  E[t] = (float)((bm[16 + t] + bm[16 + j * 16 + i]) / den);
  if (t < 16) {
    mb[t] = mu_bn[g * 16 + t];
    dmu[t] = (float)(bm[t] / den);
  }
  __syncthreads();
  for (int n = 0; n < N; ++n) {
    float* cf = coef + ((long long)n * G + g) * 528;
    cf[256 + t] += E[t];
    if (t < 16) {
      float sacc = 0.f;
      for (int k = 0; k < 16; ++k) sacc = fmaf(E[t * 16 + k], mu_in[(long long)n * C + g * 16 + k] - mb[k], sacc);
      cf[512 + t] += sacc + dmu[t];
    }
  }
}

// softmax backward of the two mixing weights: dtheta = a (da - <a, da>) = a0 a1 (da0 - da1) (1, -1)
// from the per-group differences wpart[g] = (da0 - da1, db0 - db1)
__global__ void sw_bwd_weights(const float* __restrict__ wpart, int G, const float* mean_w, const float* var_w,
                               float* dmean_w, float* dvar_w) {
  if (threadIdx.x != 0) return;
  double da = 0.0, db = 0.0;
  for (int g = 0; g < G; ++g) {
    da += wpart[g * 4 + 0];
    db += wpart[g * 4 + 1];
  }
  float a0, a1, b0, b1;
  softmax2(mean_w, a0, a1);
  softmax2(var_w, b0, b1);
  const double ca = (double)a0 * a1 * da, cb = (double)b0 * b1 * db;
  if (dmean_w) { dmean_w[0] = (float)ca; dmean_w[1] = (float)-ca; }
  if (dvar_w) { dvar_w[0] = (float)cb; dvar_w[1] = (float)-cb; }
}

// dx_p = K ge_p + L (x_p - mu_n) + c ; thread = (pixel, group)
template <typename T>
__global__ __launch_bounds__(256) void sw_bwd_apply(const T* __restrict__ gy, long long ldg, const T* __restrict__ y,
                                                    long long ldy, const T* __restrict__ x, long long ldx, int HW,
                                                    int C, int ppb, int act, const float* __restrict__ mu,
                                                    const float* __restrict__ coef, T* __restrict__ dx,
                                                    long long lddx, int accumulate) {
  extern __shared__ float sm[];  // [G][545]: K | L | c | mu
  const int n = blockIdx.y, G = C / SWC;
  for (int e = threadIdx.x; e < G * 528; e += 256)
    sm[(e / 528) * 545 + (e % 528)] = coef[(long long)n * G * 528 + e];
  for (int e = threadIdx.x; e < C; e += 256) sm[(e >> 4) * 545 + 528 + (e & 15)] = mu[(long long)n * C + e];
  __syncthreads();
  const int g = threadIdx.x % G, pl = threadIdx.x / G, rows = 256 / G;
  if (pl >= rows) return;
  const float* Km = sm + g * 545;
  const float* Lm = Km + 256;
  const float* cv = Km + 512;
  const float* mv = Km + 528;
  constexpr int V = 16 / (int)sizeof(T);
  const int p0 = blockIdx.x * ppb, p1 = min(HW, p0 + ppb);
  for (int p = p0 + pl; p < p1; p += rows) {
    const long long pp = (long long)n * HW + p;
    float ge[16], xc[16], o[16];
#pragma unroll
    for (int q = 0; q < 16; q += V) {
      ldv(gy + pp * ldg + g * 16 + q, ge + q);
      ldv(x + pp * ldx + g * 16 + q, xc + q);
    }
    if (act == 1) {
      float yv[16];
#pragma unroll
      for (int q = 0; q < 16; q += V) ldv(y + pp * ldy + g * 16 + q, yv + q);
#pragma unroll
      for (int a = 0; a < 16; ++a) ge[a] = yv[a] > 0.f ? ge[a] : 0.f;
    }
#pragma unroll
    for (int a = 0; a < 16; ++a) xc[a] -= mv[a];
    // one V-wide output chunk at a time, loop kept rolled: only V outputs and one chunk's
    // K/L rows live (fully unrolled, the hoisted LDS reads spilled ~50 VGPRs)
#pragma unroll 1
    for (int q = 0; q < 16; q += V) {
      float oc[V];
      if (accumulate) ldv(dx + pp * lddx + g * 16 + q, oc);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const int a = q + e;
        float s = cv[a];
#pragma unroll
        for (int b = 0; b < 16; ++b) s = fmaf(Km[a * 16 + b], ge[b], fmaf(Lm[a * 16 + b], xc[b], s));
        oc[e] = accumulate ? oc[e] + s : s;
      }
      stv(dx + pp * lddx + g * 16 + q, oc);
    }
    (void)o;
  }
}

// The two per-pixel 16 x 16 whitening products on the matrix cores (round 6; the thread-per-(pixel,
// group) forms above read their 16 x 16 matrices from LDS once per FMA and ran LDS-bound at 2.4-2.9
// TB/s).  A wave takes 16 pixels at a time and, for each group g, forms Y_g[16 ch][16 px] = M_g X_g
// with four v_mfma_f32_16x16x4_f32: MFMA s pairs k-slot q = lane / 16 with channel 4q + s, so lane l
// loads channels g*16 + 4q .. +3 of pixel l % 16 in one 8-B (16-bit) / 16-B (f32) load, its A
// operands are row l % 16, columns 4q .. 4q + 3 of M_g (one 16-B LDS read), and its accumulator holds
// channels 4q .. 4q + 3 of pixel l % 16 (one store).  The accumulator starts at the bias / constant
// row.  f32 products and accumulation throughout (16-bit operands are exact in f32).
template <typename T>
__global__ __launch_bounds__(256) void sw_apply_mfma(const T* __restrict__ x, long long ldx, int HW, int C, int ppb,
                                                     const float* __restrict__ aff, const float* __restrict__ bias,
                                                     int act, T* __restrict__ y, long long ldy) {
  extern __shared__ __attribute__((aligned(16))) float sm[];  // A[G][256] | b[C]
  const int n = blockIdx.y, G = C / SWC, tid = threadIdx.x;
  const f4v* an = (const f4v*)(aff + (long long)n * G * 256);
  const f4v* bn = (const f4v*)(bias + (long long)n * C);
  for (int e = tid; e < G * 64; e += 256) ((f4v*)sm)[e] = an[e];
  for (int e = tid; e < C / 4; e += 256) ((f4v*)(sm + G * 256))[e] = bn[e];
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6, pr = lane & 15, q = lane >> 4;
  const int p0 = blockIdx.x * ppb, p1 = min(HW, p0 + ppb);
  for (int pc = p0 + 16 * wave; pc < p1; pc += 64) {
    const int p = pc + pr;
    const bool ok = p < p1;
    const long long pp = (long long)n * HW + (ok ? p : p0);
    const T* xr = x + pp * ldx + 4 * q;
    T* yr = y + pp * ldy + 4 * q;
    // eight groups' loads issued before the first MFMA (one load / wait / MFMA chain / store per
    // group otherwise); a tail batch re-reads group G - 1 and stores only the groups that exist
    constexpr int GB = 8;
    for (int g0 = 0; g0 < G; g0 += GB) {
      float xv[GB][4];
#pragma unroll
      for (int j = 0; j < GB; ++j) ld4(xr + min(g0 + j, G - 1) * 16, xv[j]);
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        const int g = min(g0 + j, G - 1);
        const f4v a = *(const f4v*)(sm + g * 256 + pr * 16 + 4 * q);
        f4v acc = *(const f4v*)(sm + G * 256 + g * 16 + 4 * q);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], xv[j][s], acc, 0, 0, 0);
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (act == 1 && acc[r] < 0.f) ? 0.f : acc[r];
        if (ok && g0 + j < G) st4(yr + g * 16, o);
      }
    }
  }
}

// dx_p = K ge_p + L (x_p - mu_n) + c on the matrix cores (as sw_apply_mfma: eight MFMAs per group and
// 16 pixels, the accumulator starting at c).  Groups go four at a time with every load of the four
// issued before the first MFMA (one group per iteration, each group's loads waited for the previous
// group's MFMA chain and store: 1.05 ms over the SW step's seven launches, slower than the FMA form);
// ACT / ACC are template arguments so no branch splits the load batch.  A tail batch (G % 4) re-reads
// group G - 1 and stores only the groups that exist.
template <typename T, int ACT, int ACC>
__global__ __launch_bounds__(256) void sw_bwd_apply_mfma(const T* __restrict__ gy, long long ldg, const T* __restrict__ y,
                                                         long long ldy, const T* __restrict__ x, long long ldx, int HW,
                                                         int C, int ppb, const float* __restrict__ mu,
                                                         const float* __restrict__ coef, T* __restrict__ dx,
                                                         long long lddx) {
  extern __shared__ __attribute__((aligned(16))) float sm[];  // [G][528]: K | L | c, then mu[C]
  const int n = blockIdx.y, G = C / SWC, tid = threadIdx.x;
  const f4v* cn = (const f4v*)(coef + (long long)n * G * 528);
  for (int e = tid; e < G * 132; e += 256) ((f4v*)sm)[e] = cn[e];
  for (int e = tid; e < C / 4; e += 256) ((f4v*)(sm + G * 528))[e] = ((const f4v*)(mu + (long long)n * C))[e];
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6, pr = lane & 15, q = lane >> 4;
  const int p0 = blockIdx.x * ppb, p1 = min(HW, p0 + ppb);
  constexpr int GB = 4;
  for (int pc = p0 + 16 * wave; pc < p1; pc += 64) {
    const int p = pc + pr;
    const bool ok = p < p1;
    const long long pp = (long long)n * HW + (ok ? p : p0);
    const T* gr = gy + pp * ldg + 4 * q;
    const T* xr = x + pp * ldx + 4 * q;
    const T* yr = y + pp * ldy + 4 * q;
    T* dr = dx + pp * lddx + 4 * q;
    for (int g0 = 0; g0 < G; g0 += GB) {
      float ge[GB][4], xv[GB][4], yv[GB][4], od[GB][4];
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        const int c0 = min(g0 + j, G - 1) * 16;
        ld4(gr + c0, ge[j]);
        ld4(xr + c0, xv[j]);
        if (ACT) ld4(yr + c0, yv[j]);
        if (ACC) ld4(dr + c0, od[j]);
      }
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        const int g = min(g0 + j, G - 1);
        const float* Mg = sm + g * 528;
        const f4v mv = *(const f4v*)(sm + G * 528 + g * 16 + 4 * q);
        const f4v ka = *(const f4v*)(Mg + pr * 16 + 4 * q);
        const f4v la = *(const f4v*)(Mg + 256 + pr * 16 + 4 * q);
        f4v acc = *(const f4v*)(Mg + 512 + 4 * q);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const float gs = ACT ? (yv[j][s] > 0.f ? ge[j][s] : 0.f) : ge[j][s];
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ka[s], gs, acc, 0, 0, 0);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(la[s], xv[j][s] - mv[s], acc, 0, 0, 0);
        float o[4] = {acc[0], acc[1], acc[2], acc[3]};
        if (ACC) {
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] += od[j][r];
        }
        if (ok && g0 + j < G) st4(dr + g * 16, o);
      }
    }
  }
}

template <typename T>
void launch_sw_bwd_apply_mfma(dim3 grid, size_t lds, hipStream_t st, const T* gy, long long ldg, const T* y,
                              long long ldy, const T* x, long long ldx, int HW, int C, int ppb, int act,
                              const float* mu, const float* coef, T* dx, long long lddx, int accumulate) {
  auto k = act == 1 ? (accumulate ? sw_bwd_apply_mfma<T, 1, 1> : sw_bwd_apply_mfma<T, 1, 0>)
                    : (accumulate ? sw_bwd_apply_mfma<T, 0, 1> : sw_bwd_apply_mfma<T, 0, 0>);
  hipLaunchKernelGGL(k, grid, dim3(256), lds, st, gy, ldg, y, ldy, x, ldx, HW, C, ppb, mu, coef, dx, lddx);
}

// blocks per instance of the MFMA apply passes: ~1024 blocks over the batch, 64 .. 2048 pixels each
inline int sw_apply_nb(int HW, int N) {
  return std::max(1, std::min(dg_cdiv(HW, 64), std::max(dg_cdiv(1024, N), dg_cdiv(HW, 2048))));
}
// DGVCC_SW_APPLY=0: the thread-per-(pixel, group) apply passes (A/B; read per launch)
inline bool sw_apply_mfma_on() {
  const char* e = getenv("DGVCC_SW_APPLY");
  return !(e && e[0] == '0');
}

// pixel blocks per instance of the covariance / backward partial passes: enough blocks over the
// batch to give every CU two (the deep 48x64 layers had 3 per instance, 48 blocks in all: the
// backward partials ran at 0.3 TB/s), each at least 64 pixels, at most 64 per instance
inline int sw_nb(int HW, int N) {
  return std::max(1, std::min({64, std::max(1, HW / 64), std::max(dg_cdiv(HW, 1024), dg_cdiv(512, N))}));
}

}  // namespace

// ================================================================ C-ABI ====
extern "C" int64_t dg_iw_loss_workspace(int B, int C) {
  if (B <= 0 || C <= 0) return DG_ERR_INVALID;
  return (int64_t)B * 64 * 4;
}

extern "C" int dg_iw_loss(const float* fraw, int B, int C, float inv_hw1, float eps, const float* mask,
                          const float* num_sensitive, const float* grad_coef, float out_scale, int accumulate,
                          float* loss, float* gsym, void* workspace, void* stream) {
  DG_REQUIRE(fraw && mask && num_sensitive && B > 0 && C > 0 && (loss || gsym));
  hipStream_t st = (hipStream_t)stream;
  if (loss) {
    DG_REQUIRE(workspace);
    const int nch = std::max(1, std::min(64, dg_cdiv((long long)C * C, 4096)));
    hipLaunchKernelGGL(iw_loss_partial, dim3(nch, B), dim3(256), 0, st, fraw, C, inv_hw1, eps, mask,
                       (float*)workspace);
    DG_CHECK_LAUNCH();
    hipLaunchKernelGGL(iw_loss_finalize, dim3(1), dim3(64), 0, st, (const float*)workspace, B, nch, num_sensitive,
                       out_scale, accumulate, loss);
    DG_CHECK_LAUNCH();
  }
  if (gsym) {
    const long long total = (long long)B * C * C;
    const int grid = (int)std::min<long long>(16384, (total + 255) / 256);
    hipLaunchKernelGGL(iw_loss_grad, dim3(grid), dim3(256), 0, st, fraw, B, C, inv_hw1, eps, mask, num_sensitive,
                       grad_coef, out_scale, gsym);
    DG_CHECK_LAUNCH();
  }
  return DG_OK;
}

extern "C" int dg_iw_cov_var(const float* fraw, int B, int C, float inv_hw1, float* var, int accumulate,
                             void* stream) {
  DG_REQUIRE(fraw && var && B > 0 && C > 0);
  const long long CC = (long long)C * C;
  const int grid = (int)std::min<long long>(16384, (CC + 255) / 256);
  hipLaunchKernelGGL(iw_cov_var, dim3(grid), dim3(256), 0, (hipStream_t)stream, fraw, B, C, inv_hw1, var, accumulate);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int64_t dg_sw_save_size(int N, int C) {
  if (N <= 0 || C <= 0 || C % SWC) return DG_ERR_INVALID;
  const int64_t G = C / SWC;
  return (2 * (int64_t)N * C + 2 * (int64_t)N * G * 256 + C + G * 256) * 4;
}

extern "C" int64_t dg_sw_moments_size(int C) {
  if (C <= 0 || C % SWC) return DG_ERR_INVALID;
  return (int64_t)(C / SWC) * SW_MOM * 8;
}

static int64_t sw_ws_core(int N, int HW, int C) {  // partials + coefficients, 8-B aligned
  const int64_t G = C / SWC, nb = sw_nb(HW, N);
  const int64_t fwd = std::max<int64_t>(dg_instnorm_workspace(N, HW, C), 0) + (int64_t)N * C * 4 +
                      (int64_t)N * nb * G * 256 * 4;
  const int64_t bwd = (int64_t)N * nb * G * 272 * 4 + (int64_t)N * G * 528 * 4 + G * 4 * 4 +
                      (int64_t)N * G * SW_NP * 4;
  return (std::max(fwd, bwd) + 7) / 8 * 8;
}

// workspace of dg_sw_fwd/bwd (and of the split phases): core + one moments block
extern "C" int64_t dg_sw_workspace(int N, int HW, int C) {
  if (N <= 0 || HW <= 0 || C <= 0 || C % SWC) return DG_ERR_INVALID;
  return sw_ws_core(N, HW, C) + (int64_t)(C / SWC) * SW_MOM * 8;
}

#define SW_DISPATCH_G(KERNEL, T, ...)                                                                \
  do {                                                                                              \
    if (G <= 4)                                                                                     \
      hipLaunchKernelGGL((KERNEL<T, 1>), __VA_ARGS__);                                              \
    else if (G <= 8)                                                                                \
      hipLaunchKernelGGL((KERNEL<T, 2>), __VA_ARGS__);                                              \
    else                                                                                            \
      hipLaunchKernelGGL((KERNEL<T, 4>), __VA_ARGS__);                                              \
  } while (0)

#define SW_CHECK_SHAPE(dtype, C, T_, ...)                                                           \
  do {                                                                                              \
    DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));                                                \
    const int V_ = DG_IS16(dtype) ? 8 : 4;                                                        \
    DG_SUPPORTED(C % SWC == 0 && C <= 256 && (T_) <= SW_MAXT);                                      \
    for (int64_t ld_ : {__VA_ARGS__}) DG_SUPPORTED(ld_ % V_ == 0);                                  \
  } while (0)

// SwitchWhiten2d statistics, phase 1 (per rank): instance means/covariances into
// `save` and the batch moments [G][272] doubles into `moments`.
extern "C" int dg_sw_fwd_stats(int dtype, const void* x, int64_t ldx, int N, int HW, int C, float* save,
                               double* moments, void* workspace, void* stream) {
  DG_REQUIRE(x && save && moments && workspace && N > 0 && HW > 0 && C > 0);
  SW_CHECK_SHAPE(dtype, C, 0, ldx);
  hipStream_t st = (hipStream_t)stream;
  const int G = C / SWC, nb = sw_nb(HW, N), ppb = dg_cdiv(HW, nb);
  float* mu = save;  // mu_in is the first save slot
  char* w = (char*)workspace;
  const int64_t in_ws = dg_instnorm_workspace(N, HW, C);
  float* invstd_scratch = (float*)(w + in_ws);
  float* part = invstd_scratch + (int64_t)N * C;
  int rc = dg_instnorm_stats(dtype, x, ldx, N, HW, C, 1e-5f, mu, invstd_scratch, w, stream);
  if (rc) return rc;
  const size_t lds = (size_t)(sw_pt(C) * (C + 16) + C) * 4;
  if (dtype == DG_BF16)
    SW_DISPATCH_G(sw_cov_partial, bf16, dim3(nb, N), dim3(256), lds, st, (const bf16*)x, ldx, HW, C, ppb, mu, part);
  else if (dtype == DG_F16)
    SW_DISPATCH_G(sw_cov_partial, f16, dim3(nb, N), dim3(256), lds, st, (const f16*)x, ldx, HW, C, ppb, mu, part);
  else
    SW_DISPATCH_G(sw_cov_partial, float, dim3(nb, N), dim3(256), lds, st, (const float*)x, ldx, HW, C, ppb, mu, part);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(sw_inst_stats, dim3(G, N), dim3(256), 0, st, part, N, nb, HW, C, save);
  hipLaunchKernelGGL(sw_moments, dim3(G), dim3(256), 0, st, N, C, (const float*)save, moments);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// Phase 2: batch statistics from `moments` summed over `count` images (all ranks),
// running-stat update (training), whitening matrices, fused whiten+affine(+ReLU) apply.
extern "C" int dg_sw_fwd_finish(int dtype, const void* x, int64_t ldx, int N, int HW, int C, int T, float eps,
                                float momentum, const float* mean_w, const float* var_w, const float* gamma,
                                const float* beta, float* running_mean, float* running_cov, int training, int act,
                                int64_t count, const double* moments, float* save, void* y, int64_t ldy,
                                void* stream) {
  DG_REQUIRE(x && y && save && moments && mean_w && var_w && running_mean && running_cov && count > 0);
  DG_REQUIRE(N > 0 && HW > 0 && C > 0 && T >= 0 && (!gamma || beta));
  SW_CHECK_SHAPE(dtype, C, T, ldx, ldy);
  hipStream_t st = (hipStream_t)stream;
  const int G = C / SWC;
  hipLaunchKernelGGL(sw_finalize, dim3(G, N), dim3(256), 0, st, moments, (double)count, N, C, T, eps, momentum, mean_w,
                     var_w, gamma, beta, running_mean, running_cov, training, save);
  DG_CHECK_LAUNCH();
  const float* aff = save + (int64_t)N * C + (int64_t)N * G * 256 + C + (int64_t)G * 256;
  const float* bias = aff + (int64_t)N * G * 256;
  if (sw_apply_mfma_on()) {
    const int mnb = sw_apply_nb(HW, N);
    const int mppb = dg_cdiv(HW, mnb);
    const size_t mlds = (size_t)(G * 256 + C) * 4;
    if (dtype == DG_BF16)
      hipLaunchKernelGGL(sw_apply_mfma<bf16>, dim3(mnb, N), dim3(256), mlds, st, (const bf16*)x, ldx, HW, C, mppb, aff,
                         bias, act, (bf16*)y, ldy);
    else if (dtype == DG_F16)
      hipLaunchKernelGGL(sw_apply_mfma<f16>, dim3(mnb, N), dim3(256), mlds, st, (const f16*)x, ldx, HW, C, mppb, aff,
                         bias, act, (f16*)y, ldy);
    else
      hipLaunchKernelGGL(sw_apply_mfma<float>, dim3(mnb, N), dim3(256), mlds, st, (const float*)x, ldx, HW, C, mppb,
                         aff, bias, act, (float*)y, ldy);
    DG_CHECK_LAUNCH();
    return DG_OK;
  }
  const int anb = std::max(1, std::min(256, dg_cdiv(HW, 256)));
  const int appb = dg_cdiv(HW, anb);
  const size_t lds = (size_t)G * 273 * 4;
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(sw_apply<bf16>, dim3(anb, N), dim3(256), lds, st, (const bf16*)x, ldx, HW, C, appb, aff, bias,
                       act, (bf16*)y, ldy);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(sw_apply<f16>, dim3(anb, N), dim3(256), lds, st, (const f16*)x, ldx, HW, C, appb, aff, bias,
                       act, (f16*)y, ldy);
  else
    hipLaunchKernelGGL(sw_apply<float>, dim3(anb, N), dim3(256), lds, st, (const float*)x, ldx, HW, C, appb, aff,
                       bias, act, (float*)y, ldy);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// SwitchWhiten2d forward (sw_type 2), one rank: phase 1 + phase 2 with count = N.
// The moments live at the end of the workspace.
extern "C" int dg_sw_fwd(int dtype, const void* x, int64_t ldx, int N, int HW, int C, int T, float eps,
                         float momentum, const float* mean_w, const float* var_w, const float* gamma,
                         const float* beta, float* running_mean, float* running_cov, int training, int act,
                         float* save, void* y, int64_t ldy, void* workspace, void* stream) {
  DG_REQUIRE(workspace && N > 0 && HW > 0 && C > 0 && C % SWC == 0);
  double* moments = (double*)((char*)workspace + sw_ws_core(N, HW, C));
  int rc = dg_sw_fwd_stats(dtype, x, ldx, N, HW, C, save, moments, workspace, stream);
  if (rc) return rc;
  return dg_sw_fwd_finish(dtype, x, ldx, N, HW, C, T, eps, momentum, mean_w, var_w, gamma, beta, running_mean,
                          running_cov, training, act, N, moments, save, y, ldy, stream);
}

// Backward phase 1 (per rank): per-instance adjoints into the workspace, the batch
// adjoints (dcov_bn, dmu_bn) into `bmoments` [G][272] doubles, dgamma/dbeta.
extern "C" int dg_sw_bwd_stats(int dtype, const void* gy, int64_t ldg, const void* y, int64_t ldy, const void* x,
                               int64_t ldx, int N, int HW, int C, int T, float eps, const float* mean_w,
                               const float* var_w, const float* gamma, int act, const float* save, double* bmoments,
                               float* dgamma, float* dbeta, void* workspace, void* stream) {
  DG_REQUIRE(gy && x && save && bmoments && workspace && mean_w && var_w && (act == 0 || y));
  DG_REQUIRE(N > 0 && HW > 0 && C > 0 && T >= 0);
  SW_CHECK_SHAPE(dtype, C, T, ldx, ldg, act ? ldy : ldx);
  hipStream_t st = (hipStream_t)stream;
  const int G = C / SWC, nb = sw_nb(HW, N), ppb = dg_cdiv(HW, nb);
  const float* mu = save;
  float* part = (float*)workspace;
  float* coef = part + (int64_t)N * nb * G * 272;
  float* wpart = coef + (int64_t)N * G * 528;
  float* npart = wpart + (int64_t)G * 4;
  const size_t lds = (size_t)(2 * sw_pt(C) * (C + 16) + C) * 4;
  if (dtype == DG_BF16)
    SW_DISPATCH_G(sw_bwd_partial, bf16, dim3(nb, N), dim3(256), lds, st, (const bf16*)gy, ldg, (const bf16*)y, ldy,
                  (const bf16*)x, ldx, HW, C, ppb, act, mu, part);
  else if (dtype == DG_F16)
    SW_DISPATCH_G(sw_bwd_partial, f16, dim3(nb, N), dim3(256), lds, st, (const f16*)gy, ldg, (const f16*)y, ldy,
                  (const f16*)x, ldx, HW, C, ppb, act, mu, part);
  else
    SW_DISPATCH_G(sw_bwd_partial, float, dim3(nb, N), dim3(256), lds, st, (const float*)gy, ldg, (const float*)y, ldy,
                  (const float*)x, ldx, HW, C, ppb, act, mu, part);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(sw_bwd_small, dim3(G, N), dim3(256), 0, st, part, N, nb, HW, C, T, eps, mean_w, var_w, gamma,
                     save, coef, npart);
  hipLaunchKernelGGL(sw_bwd_reduce, dim3(G), dim3(256), 0, st, (const float*)npart, N, C, bmoments, dgamma, dbeta,
                     wpart);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// Backward phase 2: batch adjoints summed over ranks (`count` images in total) ->
// coefficients -> dx (+= when accumulate); mixing-weight gradients (this rank's part).
extern "C" int dg_sw_bwd_finish(int dtype, const void* gy, int64_t ldg, const void* y, int64_t ldy, const void* x,
                                int64_t ldx, int N, int HW, int C, int act, const float* mean_w, const float* var_w,
                                const float* save, int64_t count, const double* bmoments, void* dx, int64_t lddx,
                                int accumulate, float* dmean_w, float* dvar_w, void* workspace, void* stream) {
  DG_REQUIRE(gy && x && dx && save && bmoments && workspace && mean_w && var_w && (act == 0 || y) && count > 0);
  DG_REQUIRE(N > 0 && HW > 0 && C > 0);
  SW_CHECK_SHAPE(dtype, C, 0, ldx, ldg, lddx, act ? ldy : ldx);
  hipStream_t st = (hipStream_t)stream;
  const int G = C / SWC, nb = sw_nb(HW, N);
  const float* mu = save;
  float* part = (float*)workspace;
  float* coef = part + (int64_t)N * nb * G * 272;
  float* wpart = coef + (int64_t)N * G * 528;
  hipLaunchKernelGGL(sw_bwd_coef, dim3(G), dim3(256), 0, st, bmoments, (double)count, N, HW, C, save, coef);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(sw_bwd_weights, dim3(1), dim3(64), 0, st, wpart, G, mean_w, var_w, dmean_w, dvar_w);
  DG_CHECK_LAUNCH();
  if (sw_apply_mfma_on()) {
    const int mnb = sw_apply_nb(HW, N);
    const int mppb = dg_cdiv(HW, mnb);
    const size_t mlds = (size_t)(G * 528 + C) * 4;
    const dim3 mg(mnb, N);
    if (dtype == DG_BF16)
      launch_sw_bwd_apply_mfma<bf16>(mg, mlds, st, (const bf16*)gy, ldg, (const bf16*)y, ldy, (const bf16*)x, ldx, HW,
                                     C, mppb, act, mu, coef, (bf16*)dx, lddx, accumulate);
    else if (dtype == DG_F16)
      launch_sw_bwd_apply_mfma<f16>(mg, mlds, st, (const f16*)gy, ldg, (const f16*)y, ldy, (const f16*)x, ldx, HW, C,
                                    mppb, act, mu, coef, (f16*)dx, lddx, accumulate);
    else
      launch_sw_bwd_apply_mfma<float>(mg, mlds, st, (const float*)gy, ldg, (const float*)y, ldy, (const float*)x, ldx,
                                      HW, C, mppb, act, mu, coef, (float*)dx, lddx, accumulate);
    DG_CHECK_LAUNCH();
    return DG_OK;
  }
  const int anb = std::max(1, std::min(256, dg_cdiv(HW, 256)));
  const int appb = dg_cdiv(HW, anb);
  const size_t lds = (size_t)G * 545 * 4;
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(sw_bwd_apply<bf16>, dim3(anb, N), dim3(256), lds, st, (const bf16*)gy, ldg, (const bf16*)y, ldy,
                       (const bf16*)x, ldx, HW, C, appb, act, mu, coef, (bf16*)dx, lddx, accumulate);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(sw_bwd_apply<f16>, dim3(anb, N), dim3(256), lds, st, (const f16*)gy, ldg, (const f16*)y, ldy,
                       (const f16*)x, ldx, HW, C, appb, act, mu, coef, (f16*)dx, lddx, accumulate);
  else
    hipLaunchKernelGGL(sw_bwd_apply<float>, dim3(anb, N), dim3(256), lds, st, (const float*)gy, ldg, (const float*)y,
                       ldy, (const float*)x, ldx, HW, C, appb, act, mu, coef, (float*)dx, lddx, accumulate);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// Backward of dg_sw_fwd (training mode, one rank): phase 1 + phase 2 with count = N.
extern "C" int dg_sw_bwd(int dtype, const void* gy, int64_t ldg, const void* y, int64_t ldy, const void* x,
                         int64_t ldx, int N, int HW, int C, int T, float eps, const float* mean_w,
                         const float* var_w, const float* gamma, int act, const float* save, void* dx, int64_t lddx,
                         int accumulate, float* dgamma, float* dbeta, float* dmean_w, float* dvar_w,
                         void* workspace, void* stream) {
  DG_REQUIRE(workspace && N > 0 && HW > 0 && C > 0 && C % SWC == 0);
  double* bm = (double*)((char*)workspace + sw_ws_core(N, HW, C));
  int rc = dg_sw_bwd_stats(dtype, gy, ldg, y, ldy, x, ldx, N, HW, C, T, eps, mean_w, var_w, gamma, act, save, bm,
                           dgamma, dbeta, workspace, stream);
  if (rc) return rc;
  return dg_sw_bwd_finish(dtype, gy, ldg, y, ldy, x, ldx, N, HW, C, act, mean_w, var_w, save, N, bm, dx, lddx,
                          accumulate, dmean_w, dvar_w, workspace, stream);
}
