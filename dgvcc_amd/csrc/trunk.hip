// Elementwise/normalisation kernels of the ResNet-50 trunks (IBN-Net b, ISW, SW):
//   residual join  out = act(bn3(z) + residual)   models/ibnnet/resnet_ibn.py:96-107,
//                  models/ISW/Resnet.py:187-216, models/SW/backbones/resnet.py:100-118
//   InstanceNorm2d (affine or not) forward/backward: the IBN-b IN layers
//                  (resnet_ibn.py:77,115) and ISW's InstanceWhitening
//                  (models/ISW/instance_whitening.py:5-16)
//   ReLU backward from the saved output (torch threshold_backward semantics).
#include "dg_common.h"
#include <algorithm>
#include <cstdlib>

namespace {

constexpr int NT = 256;

inline int ew_grid(long long n) {
  long long g = (n + NT - 1) / NT;
  return (int)std::max<long long>(1, std::min<long long>(g, 16384));
}
// the channel-stationary residual join: norm.hip's cs_grid (DGVCC_EW_GRID caps the blocks)
inline int cs_grid_add(long long n) {
  // as norm.hip cs_grid (tools/bench_bn.py, profiles/round5b/bn_grid.txt): 1024 blocks
  const char* e = getenv("DGVCC_EW_GRID");
  const long long g = (n + NT - 1) / NT;
  if (e) return (int)std::max<long long>(1, std::min<long long>(g, std::max(64, atoi(e))));
  return (int)std::min<long long>(g, 1024);
}

// DGVCC_EW_UNROLL (read per launch; norm.hip's switch of the same name): 2 two pixels per loop
// trip, 1 (default) one
inline int ew_unroll() {
  const char* e = getenv("DGVCC_EW_UNROLL");
  return e && e[0] == '2' ? 2 : 1;
}

// y = act(z1*s1 + b1 + (s2 ? z2*s2 + b2 : z2)); amax (may be NULL): max |y| (the next f16 x3 convs'
// operand scales: per channel for f32, dg_common.h OutMax; zeroed by the launcher)
template <typename T, int U = 1, int NTB = NT>
__global__ __launch_bounds__(NTB) void bn_add_kernel(const T* __restrict__ z1, long long ld1, int M, int C,
                                                    const float* __restrict__ s1, const float* __restrict__ b1,
                                                    const T* __restrict__ z2, long long ld2,
                                                    const float* __restrict__ s2, const float* __restrict__ b2, int act,
                                                    T* __restrict__ y, long long ldy, float* __restrict__ amax) {
  constexpr int V = 16 / (int)sizeof(T);
  const int tpp = C / V;
  const long long gt = blockIdx.x * (long long)NTB + threadIdx.x;
  const int c0 = (int)(gt % tpp) * V;
  const long long pstride = (long long)gridDim.x * NTB / tpp;
  float a1[V], c1[V], a2[V], c2[V];
  OutMax<T, V> mx;
#pragma unroll
  for (int e = 0; e < V; e += 4) {  // 16-byte parameter loads (c0 % 4 == 0, rows 16-byte aligned)
    ld4(s1 + c0 + e, a1 + e);
    ld4(b1 + c0 + e, c1 + e);
    if (s2) {
      ld4(s2 + c0 + e, a2 + e);
      ld4(b2 + c0 + e, c2 + e);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) { a2[e + k] = 1.f; c2[e + k] = 0.f; }
    }
  }
  if constexpr (U == 1) {  // the round-3 loop (runtime flags)
    for (long long p = gt / tpp; p < M; p += pstride) {
      float u[V], v[V];
      ldv(z1 + p * ld1 + c0, u);
      ldv(z2 + p * ld2 + c0, v);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        float t = fmaf(u[e], a1[e], c1[e]) + (s2 ? fmaf(v[e], a2[e], c2[e]) : v[e]);
        if (act == 1) t = t > 0.f ? t : 0.f;
        mx.add(e, t);
        u[e] = t;
      }
      stv(y + p * ldy + c0, u);
    }
    if (amax) mx.commit(c0, C, amax);
    return;
  }
  // two pixels per trip, all four loads ahead of the first use; the second BN and the ReLU as
  // compile-time flags (straight-line bodies)
  auto run = [&](auto bn2_t, auto act_t) {
    constexpr bool BN2 = decltype(bn2_t)::value, ACT = decltype(act_t)::value;
    auto f = [&](float u[], const float v[]) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        float t = fmaf(u[e], a1[e], c1[e]) + (BN2 ? fmaf(v[e], a2[e], c2[e]) : v[e]);
        if (ACT) t = t > 0.f ? t : 0.f;
        mx.add(e, t);
        u[e] = t;
      }
    };
    long long p = gt / tpp;
    for (; p + pstride < M; p += 2 * pstride) {
      const long long q = p + pstride;
      float u0[V], v0[V], u1[V], v1[V];
      ldv(z1 + p * ld1 + c0, u0);
      ldv(z2 + p * ld2 + c0, v0);
      ldv(z1 + q * ld1 + c0, u1);
      ldv(z2 + q * ld2 + c0, v1);
      f(u0, v0);
      f(u1, v1);
      stv(y + p * ldy + c0, u0);
      stv(y + q * ldy + c0, u1);
    }
    if (p < M) {
      float u[V], v[V];
      ldv(z1 + p * ld1 + c0, u);
      ldv(z2 + p * ld2 + c0, v);
      f(u, v);
      stv(y + p * ldy + c0, u);
    }
  };
  if (s2) {
    if (act == 1) run(std::true_type{}, std::true_type{});
    else run(std::true_type{}, std::false_type{});
  } else {
    if (act == 1) run(std::false_type{}, std::true_type{});
    else run(std::false_type{}, std::false_type{});
  }
  if (amax) mx.commit(c0, C, amax);
}

// out = g * (y > 0)
template <typename T>
__global__ __launch_bounds__(NT) void relu_bwd_kernel(const T* __restrict__ g, long long ldg, const T* __restrict__ y,
                                                      long long ldy, int M, int C, T* __restrict__ out, long long ldo) {
  constexpr int V = 16 / (int)sizeof(T);
  const int tpp = C / V;
  const long long total = (long long)M * tpp;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const long long p = i / tpp;
    const int c0 = (int)(i % tpp) * V;
    float a[V], b[V];
    ldv(g + p * ldg + c0, a);
    ldv(y + p * ldy + c0, b);
#pragma unroll
    for (int e = 0; e < V; ++e) a[e] = b[e] > 0.f ? a[e] : 0.f;
    stv(out + p * ldo + c0, a);
  }
}

// ---------------------------------------------------------------- IN apply --
// Grid for the channel-stationary elementwise kernels below: gridDim.x * NT is a multiple of
// tpp = C/V, so every thread keeps one channel chunk c0 for its whole pixel loop and holds
// that chunk's per-(n, c) parameters in registers, reloading them only when n changes.
inline int cs_grid(long long total, int tpp, int nt = NT) {
  int q = tpp, a = nt;  // q = tpp / gcd(tpp, nt)
  while (a) { const int t = q % a; q = a; a = t; }
  q = tpp / q;
  // the 1024-thread form (dg_ew_wide): at most 512 blocks
  const int g = nt == NT ? ew_grid(total) : (int)std::max<long long>(1, std::min<long long>((total + nt - 1) / nt, 512));
  return (g + q - 1) / q * q;
}

// y = act((x - mu[n,c]) * is[n,c] * gamma[c] + beta[c]); amax (may be NULL): max |y|, as bn_add_kernel
template <typename T, int NTB = NT>
__global__ __launch_bounds__(NTB) void in_apply_kernel(const T* __restrict__ x, long long ldx, int N, int HW, int C,
                                                      const float* __restrict__ mu, const float* __restrict__ is,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      int act, T* __restrict__ y, long long ldy,
                                                      float* __restrict__ amax) {
  constexpr int V = 16 / (int)sizeof(T);
  const int tpp = C / V;
  const int gt = blockIdx.x * NTB + threadIdx.x;
  const int c0 = (gt % tpp) * V;
  const int pstride = gridDim.x * NTB / tpp;
  const int M = N * HW;  // M * tpp < 2^30 (checked by the ABI)
  float ga[V], be[V], m[V], s[V];
#pragma unroll
  for (int e = 0; e < V; e += 4) {  // 16-byte parameter loads (c0 % 4 == 0, rows 16-byte aligned)
    if (gamma) {
      ld4(gamma + c0 + e, ga + e);
      ld4(beta + c0 + e, be + e);
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) { ga[e + k] = 1.f; be[e + k] = 0.f; }
    }
  }
  int cur = -1;
  OutMax<T, V> mx;
  for (int p = gt / tpp; p < M; p += pstride) {
    const int n = p / HW;
    if (n != cur) {
      cur = n;
#pragma unroll
      for (int e = 0; e < V; e += 4) { ld4(mu + n * C + c0 + e, m + e); ld4(is + n * C + c0 + e, s + e); }
    }
    float v[V];
    ldv(x + p * ldx + c0, v);
#pragma unroll
    for (int e = 0; e < V; ++e) {
      float t = (v[e] - m[e]) * s[e];
      if (gamma) t = fmaf(t, ga[e], be[e]);
      if (act == 1) t = t > 0.f ? t : 0.f;
      mx.add(e, t);
      v[e] = t;
    }
    stv(y + p * ldy + c0, v);
  }
  if (amax) mx.commit(c0, C, amax);
}

// ---------------------------------------------------------------- IN bwd ----
// grid (nb, N): per (n, block) partial sums of g and g*xhat over HW
template <typename T>
__global__ __launch_bounds__(NT) void in_bwd_partial(const T* __restrict__ g, long long ldg, const T* __restrict__ x,
                                                     long long ldx, int HW, int C, int ppb, const float* __restrict__ mu,
                                                     const float* __restrict__ is, float* __restrict__ part) {
  constexpr int V = 16 / (int)sizeof(T);
  __shared__ float sh[2][NT * V];
  const int n = blockIdx.y, nb = gridDim.x;
  const int tpp = C / V, rows = NT / tpp;
  const int tid = threadIdx.x, ch = tid % tpp, pl = tid / tpp;
  const int c0 = ch * V;
  float sg[V], sx[V];
#pragma unroll
  for (int e = 0; e < V; ++e) { sg[e] = 0.f; sx[e] = 0.f; }
  const int p0 = blockIdx.x * ppb, p1 = min(HW, p0 + ppb);
  if (pl < rows) {
    float m[V], s[V];
#pragma unroll
    for (int e = 0; e < V; e += 4) { ld4(mu + n * C + c0 + e, m + e); ld4(is + n * C + c0 + e, s + e); }
    for (int p = p0 + pl; p < p1; p += rows) {
      const long long pp = (long long)n * HW + p;
      float gv[V], xv[V];
      ldv(g + pp * ldg + c0, gv);
      ldv(x + pp * ldx + c0, xv);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        sg[e] += gv[e];
        sx[e] = fmaf(gv[e], (xv[e] - m[e]) * s[e], sx[e]);
      }
    }
#pragma unroll
    for (int e = 0; e < V; ++e) { sh[0][pl * C + c0 + e] = sg[e]; sh[1][pl * C + c0 + e] = sx[e]; }
  }
  __syncthreads();
  for (int c = tid; c < C; c += NT) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < rows; ++r) { a += sh[0][r * C + c]; b += sh[1][r * C + c]; }
    float* o = part + ((long long)n * nb + blockIdx.x) * 2 * C;
    o[c] = a; o[C + c] = b;
  }
}

// coef[n][c] = (k1, k2, k3): dx = k1*g - k2*xhat - k3 ; dgamma/dbeta summed over n
// Block of FIN_CH channels x FIN_KS partial slices: the nb partials of each (n, c) are
// summed by FIN_KS threads in parallel (coalesced across c) and combined in LDS in a fixed
// order, so the result is deterministic.
constexpr int FIN_CH = 16, FIN_KS = 16;
__global__ __launch_bounds__(FIN_CH * FIN_KS) void in_bwd_finalize(const float* __restrict__ part, int N, int nb,
                                                                   int HW, int C, const float* __restrict__ is,
                                                                   const float* __restrict__ gamma, float* dgamma,
                                                                   float* dbeta, float* __restrict__ coef) {
  __shared__ double sh[2][FIN_KS][FIN_CH];
  const int cl = threadIdx.x % FIN_CH, ks = threadIdx.x / FIN_CH;
  const int c = blockIdx.x * FIN_CH + cl;
  double tg = 0.0, tx = 0.0;
  for (int n = 0; n < N; ++n) {
    double a = 0.0, b = 0.0;
    if (c < C)
      for (int k = ks; k < nb; k += FIN_KS) {
        const float* o = part + ((long long)n * nb + k) * 2 * C;
        a += o[c]; b += o[C + c];
      }
    sh[0][ks][cl] = a; sh[1][ks][cl] = b;
    __syncthreads();
    if (ks == 0 && c < C) {
      a = 0.0; b = 0.0;
      for (int r = 0; r < FIN_KS; ++r) { a += sh[0][r][cl]; b += sh[1][r][cl]; }
      tg += a; tx += b;
      const float gm = gamma ? gamma[c] : 1.f;
      const float k1 = gm * is[n * C + c];
      float* cf = coef + ((long long)n * C + c) * 3;
      cf[0] = k1;
      cf[1] = (float)(k1 * b / HW);
      cf[2] = (float)(k1 * a / HW);
    }
    __syncthreads();
  }
  if (ks == 0 && c < C) {
    if (dgamma) dgamma[c] = (float)tx;
    if (dbeta) dbeta[c] = (float)tg;
  }
}

template <typename T, int NTB = NT>
__global__ __launch_bounds__(NTB) void in_bwd_apply(const T* __restrict__ g, long long ldg, const T* __restrict__ x,
                                                   long long ldx, int N, int HW, int C, const float* __restrict__ mu,
                                                   const float* __restrict__ is, const float* __restrict__ coef,
                                                   T* __restrict__ dx, long long lddx, int accumulate,
                                                   float* __restrict__ amax) {
  constexpr int V = 16 / (int)sizeof(T);
  const int tpp = C / V;
  const int gt = blockIdx.x * NTB + threadIdx.x;
  const int c0 = (gt % tpp) * V;
  const int pstride = gridDim.x * NTB / tpp;
  const int M = N * HW;  // M * tpp < 2^30 (checked by the ABI)
  float m[V], s[V], k1[V], k2[V], k3[V];
  OutMax<T, V> mx;  // max |dx| per channel (amax, may be NULL: the following f16 x3 wgrad's operand scales)
  int cur = -1;
  for (int p = gt / tpp; p < M; p += pstride) {
    const int n = p / HW;
    if (n != cur) {
      cur = n;
      // 16-byte loads: (n C + c0) % 4 == 0, so the (k1, k2, k3) triples of the chunk start
      // 48-byte aligned
      const int nc = n * C + c0;
      float t[3 * V];
#pragma unroll
      for (int e = 0; e < V; e += 4) { ld4(mu + nc + e, m + e); ld4(is + nc + e, s + e); }
#pragma unroll
      for (int q = 0; q < 3 * V; q += 4) ld4(coef + (long long)nc * 3 + q, t + q);
#pragma unroll
      for (int e = 0; e < V; ++e) { k1[e] = t[3 * e]; k2[e] = t[3 * e + 1]; k3[e] = t[3 * e + 2]; }
    }
    float gv[V], xv[V], o[V];
    ldv(g + p * ldg + c0, gv);
    ldv(x + p * ldx + c0, xv);
    if (accumulate) ldv(dx + p * lddx + c0, o);
#pragma unroll
    for (int e = 0; e < V; ++e) {
      const float xh = (xv[e] - m[e]) * s[e];
      const float d = k1[e] * gv[e] - k2[e] * xh - k3[e];
      o[e] = accumulate ? o[e] + d : d;
      mx.add(e, o[e]);
    }
    stv(dx + p * lddx + c0, o);
  }
  if (amax) mx.commit(c0, C, amax);
}

}  // namespace

#define VOK(dtype, C, ld) ((C) % (DG_IS16(dtype) ? 8 : 4) == 0 && (ld) % (DG_IS16(dtype) ? 8 : 4) == 0)

extern "C" int dg_bn_add_apply(int dtype, const void* z1, int64_t ld1, int M, int C, const float* scale1,
                               const float* shift1, const void* z2, int64_t ld2, const float* scale2,
                               const float* shift2, int act, void* y, int64_t ldy, float* amax, void* stream) {
  DG_REQUIRE(z1 && z2 && y && scale1 && shift1 && M > 0 && C > 0 && (!scale2 || shift2));
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(VOK(dtype, C, ld1) && VOK(dtype, C, ld2) && VOK(dtype, C, ldy) && NT % (C / V) == 0);
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)M * (C / V);
  { const int zr = dg_zero_amax(amax, dtype, C, st); if (zr != DG_OK) return zr; }
  if (dtype == DG_BF16)
    hipLaunchKernelGGL((ew_unroll() == 2 ? bn_add_kernel<bf16, 2> : bn_add_kernel<bf16, 1>), dim3(cs_grid_add(total)), dim3(NT), 0, st, (const bf16*)z1, ld1, M, C, scale1,
                       shift1, (const bf16*)z2, ld2, scale2, shift2, act, (bf16*)y, ldy, amax);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL((ew_unroll() == 2 ? bn_add_kernel<f16, 2> : bn_add_kernel<f16, 1>), dim3(cs_grid_add(total)), dim3(NT), 0, st, (const f16*)z1, ld1, M, C, scale1,
                       shift1, (const f16*)z2, ld2, scale2, shift2, act, (f16*)y, ldy, amax);
  else if (dg_ew_wide(amax, true))
    hipLaunchKernelGGL((bn_add_kernel<float, 1, DG_EW_WIDE>),
                       dim3(std::max<long long>(1, std::min<long long>((total + DG_EW_WIDE - 1) / DG_EW_WIDE, 256))),
                       dim3(DG_EW_WIDE), 0, st, (const float*)z1, ld1, M, C, scale1, shift1, (const float*)z2, ld2,
                       scale2, shift2, act, (float*)y, ldy, amax);
  else
    hipLaunchKernelGGL((ew_unroll() == 2 ? bn_add_kernel<float, 2> : bn_add_kernel<float, 1>), dim3(cs_grid_add(total)), dim3(NT), 0, st, (const float*)z1, ld1, M, C,
                       scale1, shift1, (const float*)z2, ld2, scale2, shift2, act, (float*)y, ldy, amax);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_relu_bwd(int dtype, const void* g, int64_t ldg, const void* y, int64_t ldy, int M, int C, void* out,
                           int64_t ldo, void* stream) {
  DG_REQUIRE(g && y && out && M > 0 && C > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(VOK(dtype, C, ldg) && VOK(dtype, C, ldy) && VOK(dtype, C, ldo));
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)M * (C / V);
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(relu_bwd_kernel<bf16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const bf16*)g, ldg,
                       (const bf16*)y, ldy, M, C, (bf16*)out, ldo);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(relu_bwd_kernel<f16>, dim3(ew_grid(total)), dim3(NT), 0, st, (const f16*)g, ldg,
                       (const f16*)y, ldy, M, C, (f16*)out, ldo);
  else
    hipLaunchKernelGGL(relu_bwd_kernel<float>, dim3(ew_grid(total)), dim3(NT), 0, st, (const float*)g, ldg,
                       (const float*)y, ldy, M, C, (float*)out, ldo);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_instnorm_apply(int dtype, const void* x, int64_t ldx, int N, int HW, int C, const float* mean,
                                 const float* invstd, const float* gamma, const float* beta, int act, void* y,
                                 int64_t ldy, float* amax, void* stream) {
  DG_REQUIRE(x && y && mean && invstd && N > 0 && HW > 0 && C > 0 && (!gamma || beta));
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  const int V = DG_IS16(dtype) ? 8 : 4;
  const long long total = (long long)N * HW * (C / V);
  DG_SUPPORTED(VOK(dtype, C, ldx) && VOK(dtype, C, ldy) && total < (1LL << 30));
  hipStream_t st = (hipStream_t)stream;
  const int grid = cs_grid(total, C / V);
  { const int zr = dg_zero_amax(amax, dtype, C, st); if (zr != DG_OK) return zr; }
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(in_apply_kernel<bf16>, dim3(grid), dim3(NT), 0, st, (const bf16*)x, ldx, N, HW, C,
                       mean, invstd, gamma, beta, act, (bf16*)y, ldy, amax);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(in_apply_kernel<f16>, dim3(grid), dim3(NT), 0, st, (const f16*)x, ldx, N, HW, C,
                       mean, invstd, gamma, beta, act, (f16*)y, ldy, amax);
  else if (dg_ew_wide(amax, true))
    hipLaunchKernelGGL((in_apply_kernel<float, DG_EW_WIDE>), dim3(cs_grid(total, C / V, DG_EW_WIDE)), dim3(DG_EW_WIDE),
                       0, st, (const float*)x, ldx, N, HW, C, mean, invstd, gamma, beta, act, (float*)y, ldy, amax);
  else
    hipLaunchKernelGGL(in_apply_kernel<float>, dim3(grid), dim3(NT), 0, st, (const float*)x, ldx, N, HW, C,
                       mean, invstd, gamma, beta, act, (float*)y, ldy, amax);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

static inline int in_nb(int HW) { return std::max(1, std::min(64, dg_cdiv(HW, 256))); }

extern "C" int64_t dg_instnorm_bwd_workspace(int N, int HW, int C) {
  if (N <= 0 || HW <= 0 || C <= 0) return DG_ERR_INVALID;
  return ((int64_t)N * in_nb(HW) * 2 * C + (int64_t)N * C * 3) * 4;
}

// g: upstream gradient already masked by any following ReLU; dgamma/dbeta may be NULL
extern "C" int dg_instnorm_bwd(int dtype, const void* g, int64_t ldg, const void* x, int64_t ldx, int N, int HW, int C,
                               const float* mean, const float* invstd, const float* gamma, void* dx, int64_t lddx,
                               int accumulate, float* dgamma, float* dbeta, void* workspace, float* amax,
                               void* stream) {
  DG_REQUIRE(g && x && dx && mean && invstd && workspace && N > 0 && HW > 0 && C > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  const int V = DG_IS16(dtype) ? 8 : 4;
  const long long total = (long long)N * HW * (C / V);
  DG_SUPPORTED(VOK(dtype, C, ldg) && VOK(dtype, C, ldx) && VOK(dtype, C, lddx) && C / V <= NT &&
               total < (1LL << 30));
  hipStream_t st = (hipStream_t)stream;
  const int nb = in_nb(HW), ppb = dg_cdiv(HW, nb);
  float* part = (float*)workspace;
  float* coef = part + (long long)N * nb * 2 * C;
  const int grid = cs_grid(total, C / V);
  const dim3 fgrid(dg_cdiv(C, FIN_CH)), fblk(FIN_CH * FIN_KS);
  { const int zr = dg_zero_amax(amax, dtype, C, st); if (zr != DG_OK) return zr; }
  if (dtype == DG_BF16) {
    hipLaunchKernelGGL(in_bwd_partial<bf16>, dim3(nb, N), dim3(NT), 0, st, (const bf16*)g, ldg, (const bf16*)x, ldx,
                       HW, C, ppb, mean, invstd, part);
    DG_CHECK_LAUNCH();
    hipLaunchKernelGGL(in_bwd_finalize, fgrid, fblk, 0, st, part, N, nb, HW, C, invstd, gamma, dgamma, dbeta, coef);
    DG_CHECK_LAUNCH();
    hipLaunchKernelGGL(in_bwd_apply<bf16>, dim3(grid), dim3(NT), 0, st, (const bf16*)g, ldg, (const bf16*)x,
                       ldx, N, HW, C, mean, invstd, coef, (bf16*)dx, lddx, accumulate, amax);
  } else if (dtype == DG_F16) {
    hipLaunchKernelGGL(in_bwd_partial<f16>, dim3(nb, N), dim3(NT), 0, st, (const f16*)g, ldg, (const f16*)x, ldx,
                       HW, C, ppb, mean, invstd, part);
    DG_CHECK_LAUNCH();
    hipLaunchKernelGGL(in_bwd_finalize, fgrid, fblk, 0, st, part, N, nb, HW, C, invstd, gamma, dgamma, dbeta, coef);
    DG_CHECK_LAUNCH();
    hipLaunchKernelGGL(in_bwd_apply<f16>, dim3(grid), dim3(NT), 0, st, (const f16*)g, ldg, (const f16*)x,
                       ldx, N, HW, C, mean, invstd, coef, (f16*)dx, lddx, accumulate, amax);
  } else {
    hipLaunchKernelGGL(in_bwd_partial<float>, dim3(nb, N), dim3(NT), 0, st, (const float*)g, ldg, (const float*)x,
                       ldx, HW, C, ppb, mean, invstd, part);
    DG_CHECK_LAUNCH();
    hipLaunchKernelGGL(in_bwd_finalize, fgrid, fblk, 0, st, part, N, nb, HW, C, invstd, gamma, dgamma, dbeta, coef);
    DG_CHECK_LAUNCH();
    if (dg_ew_wide(amax, true))
      hipLaunchKernelGGL((in_bwd_apply<float, DG_EW_WIDE>), dim3(cs_grid(total, C / V, DG_EW_WIDE)),
                         dim3(DG_EW_WIDE), 0, st, (const float*)g, ldg, (const float*)x, ldx, N, HW, C, mean, invstd,
                         coef, (float*)dx, lddx, accumulate, amax);
    else
      hipLaunchKernelGGL(in_bwd_apply<float>, dim3(grid), dim3(NT), 0, st, (const float*)g, ldg,
                         (const float*)x, ldx, N, HW, C, mean, invstd, coef, (float*)dx, lddx, accumulate, amax);
  }
  DG_CHECK_LAUNCH();
  return DG_OK;
}
