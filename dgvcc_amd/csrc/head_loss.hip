// Density head (1x1 conv C->1 + act), MSE loss, fused AdamW, flat gather and
// the Gaussian density-map scatter.
//   den_head            models/models.py:60-62  (ConvBlock(256,1,k=1), ReLU)
//   cls_head tail       models/models.py:241-243 (Conv1x1 256->1 + Sigmoid)
//   MSELoss             trainers/dgtrainer.py:57
//   AdamW               main.py:85-86 (torch.optim.AdamW semantics)
//   dmap scatter        utils/dmap_gen.py:53-81 (gaussian_filter_density_fixed)
#include "dg_common.h"
#include <cmath>
#include <algorithm>

namespace {

constexpr int NT = 256;

inline int ew_grid(long long n, int cap = 8192) {
  long long g = (n + NT - 1) / NT;
  return (int)std::max<long long>(1, std::min<long long>(g, cap));
}

// ---------------------------------------------------------------- head -----
// TPP threads cooperate on one pixel (V channels each), xor-shuffle reduce.
template <typename T, int TPP>
__global__ __launch_bounds__(NT) void head_fwd_kernel(const T* __restrict__ x, long long ldx, int M, int C,
                                                      const float* __restrict__ w, const float* bias, int act,
                                                      float* __restrict__ y) {
  constexpr int V = 16 / (int)sizeof(T);
  constexpr int PPB = NT / TPP;
  const int lane = threadIdx.x % TPP;
  for (long long p0 = (long long)blockIdx.x * PPB; p0 < M; p0 += (long long)gridDim.x * PPB) {
    const long long p = p0 + threadIdx.x / TPP;
    float s = 0.f;
    if (p < M) {
      for (int c = lane * V; c < C; c += TPP * V) {
        float v[V];
        ldv(x + p * ldx + c, v);
#pragma unroll
        for (int e = 0; e < V; ++e) s = fmaf(v[e], w[c + e], s);
      }
    }
#pragma unroll
    for (int o = TPP / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (p < M && lane == 0) {
      if (bias) s += bias[0];
      if (act == 1) s = s > 0.f ? s : 0.f;
      else if (act == 2) s = 1.f / (1.f + expf(-s));
      y[p] = s;
    }
  }
}

__device__ __forceinline__ float head_gpre(float gy, float y, int act) {
  if (act == 1) return y > 0.f ? gy : 0.f;
  if (act == 2) return gy * y * (1.f - y);
  return gy;
}

// gx[p][c] = gpre[p] * w[c];  partial gw[blk][c] = sum_p gpre[p] * x[p][c]
template <typename T>
__global__ __launch_bounds__(NT) void head_bwd_kernel(const T* __restrict__ x, long long ldx, int M, int C,
                                                      const float* __restrict__ w, int act, const float* __restrict__ y,
                                                      const float* __restrict__ gy, T* gx, long long ldgx, int acc_gx,
                                                      int ppb, float* __restrict__ part) {
  constexpr int V = 16 / (int)sizeof(T);
  __shared__ float sh[NT * V + NT];
  const int tpp = C / V, rows = NT / tpp;
  const int tid = threadIdx.x, ch = tid % tpp, pl = tid / tpp;
  const int c0 = ch * V;
  float s[V], sb = 0.f;
#pragma unroll
  for (int e = 0; e < V; ++e) s[e] = 0.f;
  const int p0 = blockIdx.x * ppb, p1 = min(M, p0 + ppb);
  if (pl < rows) {
    float wv[V];
#pragma unroll
    for (int e = 0; e < V; ++e) wv[e] = w[c0 + e];
    for (int p = p0 + pl; p < p1; p += rows) {
      const float g = head_gpre(gy[p], y[p], act);
      float v[V];
      ldv(x + (long long)p * ldx + c0, v);
#pragma unroll
      for (int e = 0; e < V; ++e) s[e] = fmaf(g, v[e], s[e]);
      if (ch == 0) sb += g;
      if (gx) {
        float o[V];
        if (acc_gx) ldv(gx + (long long)p * ldgx + c0, o);
        else {
#pragma unroll
          for (int e = 0; e < V; ++e) o[e] = 0.f;
        }
#pragma unroll
        for (int e = 0; e < V; ++e) o[e] = fmaf(g, wv[e], o[e]);
        stv(gx + (long long)p * ldgx + c0, o);
      }
    }
#pragma unroll
    for (int e = 0; e < V; ++e) sh[pl * C + c0 + e] = s[e];
  }
  sh[NT * V + tid] = sb;
  __syncthreads();
  for (int c = tid; c < C; c += NT) {
    float a = 0.f;
    for (int r = 0; r < rows; ++r) a += sh[r * C + c];
    part[(long long)blockIdx.x * (C + 1) + c] = a;
  }
  if (tid == 0) {
    float b = 0.f;
    for (int r = 0; r < NT; ++r) b += sh[NT * V + r];
    part[(long long)blockIdx.x * (C + 1) + C] = b;
  }
}

// One block per column: 256 threads stride the rows, then a fixed-order tree (deterministic).
__global__ __launch_bounds__(NT) void colsum_kernel(const float* __restrict__ part, int nblk, int ncol, float* out0,
                                                    int n0, float* out1) {
  __shared__ double sh[NT];
  const int c = blockIdx.x;
  double a = 0.0;
  for (int k = threadIdx.x; k < nblk; k += NT) a += part[(long long)k * ncol + c];
  sh[threadIdx.x] = a;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  if (c < n0) out0[c] = (float)sh[0];
  else if (out1) out1[c - n0] = (float)sh[0];
}

inline int head_nblk(int M) { return std::max(1, std::min(1024, dg_cdiv(M, 64))); }

// ---------------------------------------------------------------- MSE ------
__global__ __launch_bounds__(NT) void mse_partial(const float* __restrict__ pred, const float* __restrict__ gt,
                                                  float gs, long long n, float* __restrict__ dpred, float gcoef,
                                                  float* __restrict__ part) {
  __shared__ float sh[NT / 64];
  float s = 0.f;
  const float k = 2.f * gcoef / (float)n;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const float d = pred[i] - gt[i] * gs;
    s = fmaf(d, d, s);
    if (dpred) dpred[i] = k * d;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < NT / 64; ++i) t += sh[i];
    part[blockIdx.x] = t;
  }
}

// launched as one block of >= 64 threads; wave 0 reduces: lane-strided double sums + fixed xor tree
__global__ void mse_final(const float* __restrict__ part, int nblk, long long n, float* loss) {
  if (threadIdx.x >= 64) return;
  double a = 0.0;
  for (int i = threadIdx.x; i < nblk; i += 64) a += part[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
  if (threadIdx.x == 0) loss[0] = (float)(a / (double)n);
}

// ---------------------------------------------------------------- BCE ------
// F.binary_cross_entropy (mean): -(t*max(log p,-100) + (1-t)*max(log(1-p),-100));
// grad = (p - t) / max((1-p)*p, 1e-12) / n   (ATen binary_cross_entropy_backward)
__global__ __launch_bounds__(NT) void bce_partial(const float* __restrict__ p, const float* __restrict__ t,
                                                  long long n, float* __restrict__ dp, float gcoef,
                                                  float* __restrict__ part) {
  __shared__ float sh[NT / 64];
  float s = 0.f;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    const float pi = p[i], ti = t[i];
    const float lp = fmaxf(logf(pi), -100.f), l1p = fmaxf(logf(1.f - pi), -100.f);
    s -= ti * lp + (1.f - ti) * l1p;
    if (dp) dp[i] = gcoef * (pi - ti) / fmaxf((1.f - pi) * pi, 1e-12f) / (float)n;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f;
    for (int i = 0; i < NT / 64; ++i) a += sh[i];
    part[blockIdx.x] = a;
  }
}

// ---------------------------------------------------------------- AdamW ----
__global__ __launch_bounds__(NT) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, long long n, float lr,
                                                   float b1, float b2, float eps, float wd, float step_size,
                                                   float bc2_sqrt) {
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT) {
    float pi = p[i];
    const float gi = g[i];
    pi *= 1.f - lr * wd;
    float mi = m[i];
    mi = fmaf(1.f - b1, gi - mi, mi);  // exp_avg.lerp_(grad, 1 - beta1)
    float vi = v[i] * b2;
    vi = fmaf((1.f - b2) * gi, gi, vi);  // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi - step_size * (mi / denom);
    p[i] = pi; m[i] = mi; v[i] = vi;
  }
}

// One block per GATHER_CHUNK elements of the flat buffer: the block finds the tensor holding its first
// element (binary search over the offsets, uniform) and copies the chunk tensor by tensor.  The earlier
// grid of 64 blocks per tensor left the large tensors (2.4M elements) to 16k threads looping over
// dependent 4-B copies: 0.13 ms for the ResNet-50 gradients, ~1 TB/s.
constexpr int GATHER_CHUNK = 4096;
__global__ __launch_bounds__(NT) void gather_flat_kernel(const float* const* __restrict__ ptrs,
                                                         const int64_t* __restrict__ offsets, int count,
                                                         float* __restrict__ flat) {
  const long long c0 = blockIdx.x * (long long)GATHER_CHUNK;
  if (c0 >= offsets[count]) return;
  const long long c1 = min((long long)offsets[count], c0 + GATHER_CHUNK);
  int lo = 0, hi = count - 1;  // last tensor starting at or before c0
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (offsets[mid] <= c0) lo = mid;
    else hi = mid - 1;
  }
  for (int t = lo; t < count && offsets[t] < c1; ++t) {
    const long long o = offsets[t];
    const long long b = max(o, c0), e = min((long long)offsets[t + 1], c1);
    const float* src = ptrs[t];
#pragma unroll 4
    for (long long i = b + threadIdx.x; i < e; i += NT) flat[i] = src[i - o];
  }
}

// ---------------------------------------------------------------- dmap -----
// One wave per point: lane l < 225 handles stamp cell (l/15, l%15) — 4 passes.
__global__ void dmap_fixed_kernel(const float* __restrict__ pts, const int64_t* __restrict__ offsets, int N, int H,
                                  int W, float sigma, int radius, float* __restrict__ dmap) {
  __shared__ float wts[64];
  const int K = 2 * radius + 1;
  if (threadIdx.x < K) {
    // scipy.ndimage._gaussian_kernel1d in float64, then the per-axis float32 output
    double s = 0.0;
    for (int i = -radius; i <= radius; ++i) s += exp(-0.5 / ((double)sigma * sigma) * (double)(i * i));
    const int i = threadIdx.x - radius;
    wts[threadIdx.x] = (float)(exp(-0.5 / ((double)sigma * sigma) * (double)(i * i)) / s);
  }
  __syncthreads();
  __shared__ double wd[64];
  if (threadIdx.x < K) {
    double s = 0.0;
    for (int i = -radius; i <= radius; ++i) s += exp(-0.5 / ((double)sigma * sigma) * (double)(i * i));
    const int i = threadIdx.x - radius;
    wd[threadIdx.x] = exp(-0.5 / ((double)sigma * sigma) * (double)(i * i)) / s;
  }
  __syncthreads();
  const long long total = offsets[N];
  const int waves = blockDim.x / 64, lane = threadIdx.x & 63;
  for (long long q = (long long)blockIdx.x * waves + (threadIdx.x >> 6); q < total; q += (long long)gridDim.x * waves) {
    // image index of point q (binary search over offsets)
    int lo = 0, hi = N;
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (offsets[mid] <= q) lo = mid; else hi = mid;
    }
    const int n = lo;
    const float px = pts[2 * q], py = pts[2 * q + 1];
    // int() truncation; negative indices wrap like numpy (dmap_gen.py:74-75)
    int r = (int)py, c = (int)px;
    if (!(r < H && c < W)) continue;
    if (r < 0) r += H;
    if (c < 0) c += W;
    if (r < 0 || c < 0) continue;
    float* img = dmap + (long long)n * H * W;
    for (int cell = lane; cell < K * K; cell += 64) {
      const int di = cell / K, dj = cell % K;
      const int rr = r + di - radius, cc = c + dj - radius;
      if ((unsigned)rr < (unsigned)H && (unsigned)cc < (unsigned)W) {
        const float v = (float)((double)wts[di] * wd[dj]);
        atomicAdd(img + (long long)rr * W + cc, v);
      }
    }
  }
}

// ---------------------------------------------------------------- adaptive dmap
// utils/dmap_gen.py:14-51: sigma_i = 0.1 * (d1 + d2 + d3) over the 4 nearest
// points (KDTree query k=4 includes the point itself; duplicates count as 0),
// sigma = 15 when the image has <= 3 points; truncate 4 -> radius int(4 sigma + 0.5).
__global__ void knn_sigma_kernel(const float* __restrict__ pts, const int64_t* __restrict__ offsets, int N,
                                 double* __restrict__ sigma) {
  const long long total = offsets[N];
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < total;
       q += (long long)gridDim.x * blockDim.x) {
    int lo = 0, hi = N;
    while (hi - lo > 1) { const int mid = (lo + hi) >> 1; if (offsets[mid] <= q) lo = mid; else hi = mid; }
    const long long p0 = offsets[lo], p1 = offsets[lo + 1];
    if (p1 - p0 <= 3) { sigma[q] = 15.0; continue; }
    const double x = pts[2 * q], y = pts[2 * q + 1];
    double d[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
    for (long long j = p0; j < p1; ++j) {
      const double dx = (double)pts[2 * j] - x, dy = (double)pts[2 * j + 1] - y;
      double v = sqrt(dx * dx + dy * dy);
      if (v < d[3]) {  // insertion into the sorted 4 smallest
        int k = 3;
        while (k > 0 && d[k - 1] > v) { d[k] = d[k - 1]; --k; }
        d[k] = v;
      }
    }
    sigma[q] = (d[1] + d[2] + d[3]) * 0.1;
  }
}

// one block per point: separable stamp of radius int(4 sigma + 0.5), clipped
__global__ __launch_bounds__(NT) void dmap_adaptive_kernel(const float* __restrict__ pts,
                                                           const int64_t* __restrict__ offsets, int N, int H, int W,
                                                           const double* __restrict__ sigma, float* __restrict__ dmap) {
  __shared__ double wd[2048];
  __shared__ float wf[2048];
  __shared__ double ssum;
  const long long total = offsets[N];
  for (long long q = blockIdx.x; q < total; q += gridDim.x) {
    int lo = 0, hi = N;
    while (hi - lo > 1) { const int mid = (lo + hi) >> 1; if (offsets[mid] <= q) lo = mid; else hi = mid; }
    const float px = pts[2 * q], py = pts[2 * q + 1];
    int r = (int)py, c = (int)px;
    if (!(r < H && c < W)) continue;  // uniform per block
    if (r < 0) r += H;
    if (c < 0) c += W;
    if (r < 0 || c < 0) continue;
    const double sg = sigma[q];
    int rad = (int)(4.0 * sg + 0.5);
    if (rad > 1023) rad = 1023;
    const int K = 2 * rad + 1;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = 0.0;
      for (int i = -rad; i <= rad; ++i) s += exp(-0.5 / (sg * sg) * (double)i * i);
      ssum = s;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < K; i += blockDim.x) {
      const double v = exp(-0.5 / (sg * sg) * (double)(i - rad) * (i - rad)) / ssum;
      wd[i] = v;
      wf[i] = (float)v;
    }
    __syncthreads();
    // only the in-frame part of the stamp
    const int r0 = max(0, r - rad), r1 = min(H, r + rad + 1);
    const int c0 = max(0, c - rad), c1 = min(W, c + rad + 1);
    const int cw = c1 - c0;
    float* img = dmap + (long long)lo * H * W;
    const long long cells = (long long)(r1 - r0) * cw;
    for (long long t = threadIdx.x; t < cells; t += blockDim.x) {
      const int rr = r0 + (int)(t / cw), cc = c0 + (int)(t % cw);
      const float v = (float)((double)wf[rr - r + rad] * wd[cc - c + rad]);
      atomicAdd(img + (long long)rr * W + cc, v);
    }
  }
}

// Deterministic variant (no atomics on the map): every output pixel sums its stamp values in
// point order, the reference's `density += gaussian_filter(pt2d)` f32 accumulation
// (dmap_gen.py:72-79) exactly, so the map is bit-identical to the reference's and stable run
// to run.  One launch, one 256-thread block per 64 x 64 output tile: the block first forms the
// normalized 1-D weights (scipy's float64 kernel, dmap_gen.py's gaussian_filter) in LDS, then walks
// its image's points in order, 256 at a time: each thread tests one point's stamp against the
// tile, the hits are compacted in point order (wave ballots + an LDS prefix over the 4 waves), and
// every thread adds the hits' stamp values -- (float)(wf[di] * wd[dj]), scipy's two float32 passes
// -- to its 4 x 4 pixels.  No stamp table, no binning pass, no scan, no atomics: the point list of
// an image (8 B per point) is read once per tile from L2, the map written once with 16-B stores.
// Measured against the alternatives (16 frames of 768 x 1024, ~490 points each, HIP-graph
// replay): 19.8 us here; 128 x 64 tiles (half the blocks, one CU-slot round) 27.1 us; one
// barrier-free wave per 32 x 64 strip (ballot + lane-permute walk of every point) 24.9 us; the
// earlier stamp-table launch + 32 x 64 tiles 20.7 us.
// int() truncation and numpy's negative-index wrap of gaussian_filter_density_fixed
__device__ __forceinline__ bool dm_coords(float x, float y, int H, int W, int& r, int& c) {
  r = (int)y;
  c = (int)x;
  const bool in = r < H && c < W;
  if (r < 0) r += H;
  if (c < 0) c += W;
  return in && r >= 0 && c >= 0;
}
__device__ __forceinline__ bool dm_point(const float* __restrict__ pts, long long q, int H, int W, int& r, int& c) {
  r = (int)pts[2 * q + 1];
  c = (int)pts[2 * q];
  const bool in = r < H && c < W;
  if (r < 0) r += H;
  if (c < 0) c += W;
  return in && r >= 0 && c >= 0;
}

// DFR x DFC tiles, 4 columns per thread (one 16-B store per row), DFC / 4 threads per row,
// rows strided by 256 / (DFC / 4) within a thread; PF: the first chunk's point loaded before the weights.
// PERS = 1: a grid of at most DMAP_PERS_BLOCKS blocks walks the (image, tile) list, so the weights are
// formed once per block and a tile's point scan overlaps the previous tile's stores (which the block
// does not wait for); the tile math and the per-pixel summation order are unchanged (bit-identical).
constexpr int DMAP_PERS_BLOCKS = 1024;
// HOSTW = 1: the normalized 1-D weights formed once on the host by the launcher (the same float64
// expressions in the same order, glibc's exp as numpy's) and passed by value, so a block only copies
// them into LDS: no per-block exp / normalization chain and one barrier fewer ahead of the point walk
struct DmapWeights {
  double wd[64];
  float wf[64];
};
// PTS = 2: chunks of 512 points, two per thread (both loads issued before the first test; the hits of
// the first 256 compacted ahead of the second's, so still in point order): one chunk's three barriers
// for an image of up to 512 points instead of two chunks'
template <int DFR, int PF, int DFC = 64, int PERS = 0, int HOSTW = 0, int PTS = 1>
__global__ __launch_bounds__(256) void dmap_fixed_fused_kernel(const float* __restrict__ pts,
                                                               const int64_t* __restrict__ offsets, int H, int W,
                                                               float sigma, int radius, float* __restrict__ dmap,
                                                               int nimg, DmapWeights hw) {
  static_assert(PTS == 1 || !PF, "PTS 2: without the prefetched first chunk");
  __shared__ double ex[64], wd[64];
  __shared__ float wf[64];
  __shared__ int hr[256 * PTS], hc[256 * PTS];
  __shared__ int wcnt[4 * PTS];
  const int K = 2 * radius + 1;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid < K) {
    if (HOSTW) {
      wd[tid] = hw.wd[tid];
      wf[tid] = hw.wf[tid];
    } else {
      const int i = tid - radius;
      ex[tid] = exp(-0.5 / ((double)sigma * sigma) * (double)(i * i));
    }
  }
  const int tiles_w = (W + DFC - 1) / DFC;
  const int tiles = ((H + DFR - 1) / DFR) * tiles_w;
  constexpr int TPR = DFC / 4, RPP = 256 / TPR, RT = DFR / RPP;
  const long long tot = PERS ? (long long)tiles * nimg : 1;
  long long it = PERS ? blockIdx.x : 0;
  bool first = true;
  for (; it < tot; it += PERS ? gridDim.x : 1) {
  const int bt = PERS ? (int)(it % tiles) : blockIdx.x;
  const int n = PERS ? (int)(it / tiles) : blockIdx.y;
  const int ty0 = (bt / tiles_w) * DFR, tx0 = (bt % tiles_w) * DFC;
  const int pr = ty0 + tid / TPR, pc = tx0 + (tid % TPR) * 4;  // pixels (pr + a RPP, pc..pc+3), a < RT
  const long long p0 = offsets[n], p1 = offsets[n + 1];
  float fx = 0.f, fy = 0.f;
  if (PF && p0 + tid < p1) {
    fx = pts[2 * (p0 + tid)];
    fy = pts[2 * (p0 + tid) + 1];
  }
  if (!HOSTW && first) {
    __syncthreads();
    if (tid < K) {  // phi / phi.sum(), summed in index order
      double s = 0.0;
      for (int j = 0; j < K; ++j) s += ex[j];
      wd[tid] = ex[tid] / s;
      wf[tid] = (float)wd[tid];
    }
    first = false;
  }
  float acc[RT][4] = {};
  for (long long base = p0; base < p1; base += 256 * PTS) {
    int tot4 = 0;
    if constexpr (PTS > 1) {
      int rr[PTS], cc[PTS];
      bool ht[PTS];
#pragma unroll
      for (int u = 0; u < PTS; ++u) {
        const long long q = base + u * 256 + tid;
        ht[u] = false;
        rr[u] = cc[u] = 0;
        if (q < p1 && dm_point(pts, q, H, W, rr[u], cc[u]))
          ht[u] = rr[u] + radius >= ty0 && rr[u] - radius < ty0 + DFR && cc[u] + radius >= tx0 && cc[u] - radius < tx0 + DFC;
      }
      unsigned long long mm[PTS];
#pragma unroll
      for (int u = 0; u < PTS; ++u) {
        mm[u] = __ballot(ht[u]);
        if (lane == 0) wcnt[u * 4 + wv] = __popcll(mm[u]);
      }
      __syncthreads();  // also publishes the weights on the first pass
      int offu[PTS];
#pragma unroll
      for (int u = 0; u < PTS; ++u) {
        int before = 0, all = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          before += w < wv ? wcnt[u * 4 + w] : 0;
          all += wcnt[u * 4 + w];
        }
        offu[u] = tot4 + before;
        tot4 += all;
      }
#pragma unroll
      for (int u = 0; u < PTS; ++u)
        if (ht[u]) {
          const int k = offu[u] + __popcll(mm[u] & ((1ull << lane) - 1ull));
          hr[k] = rr[u];
          hc[k] = cc[u];
        }
      __syncthreads();
    } else {
    const long long q = base + tid;
    int r = 0, c = 0;
    bool hit = false;
    if (PF) {
      if (q < p1) {
        const float x = fx, y = fy;
        if (q + 256 < p1) {
          fx = pts[2 * (q + 256)];
          fy = pts[2 * (q + 256) + 1];
        }
        if (dm_coords(x, y, H, W, r, c))
          hit = r + radius >= ty0 && r - radius < ty0 + DFR && c + radius >= tx0 && c - radius < tx0 + DFC;
      }
    } else if (q < p1 && dm_point(pts, q, H, W, r, c)) {
      hit = r + radius >= ty0 && r - radius < ty0 + DFR && c + radius >= tx0 && c - radius < tx0 + DFC;
    }
    const unsigned long long m = __ballot(hit);
    if (lane == 0) wcnt[wv] = __popcll(m);
    __syncthreads();  // also publishes the weights on the first pass
    int off = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      off += w < wv ? wcnt[w] : 0;
      tot4 += wcnt[w];
    }
    if (hit) {
      const int k = off + __popcll(m & ((1ull << lane) - 1ull));
      hr[k] = r;
      hc[k] = c;
    }
    __syncthreads();
    }
    for (int j = 0; j < tot4; ++j) {  // the hits in point order
      const int di0 = pr - hr[j] + radius, dj0 = pc - hc[j] + radius;
      if (di0 + (RT - 1) * RPP < 0 || di0 >= K || dj0 + 3 < 0 || dj0 >= K) continue;
#pragma unroll
      for (int a = 0; a < RT; ++a) {
        const int di = di0 + a * RPP;
        if ((unsigned)di >= (unsigned)K) continue;
        const double f = (double)wf[di];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int dj = dj0 + k;
          if ((unsigned)dj < (unsigned)K) acc[a][k] += (float)(f * wd[dj]);
        }
      }
    }
    __syncthreads();  // hr / hc / wcnt are rewritten by the next chunk
  }
  if (p0 >= p1 && PERS) __syncthreads();  // no chunk ran: the weights still need their barrier
#pragma unroll
  for (int a = 0; a < RT; ++a) {
    if (pr + a * RPP >= H) continue;
    float* o = dmap + ((long long)n * H + pr + a * RPP) * W + pc;
    if (pc + 3 < W && (W & 3) == 0) {
      *(f4v*)o = f4v{acc[a][0], acc[a][1], acc[a][2], acc[a][3]};
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (pc + k < W) o[k] = acc[a][k];
    }
  }
  }
}

// fp16 mode loss scaling: g *= inv_scale in place; any non-finite element sets *nonfinite = 1
// (plain vector stores of the same value; the flag is zeroed by the caller)
__global__ void grad_unscale_kernel(float* __restrict__ g, long long n, float inv_scale, int* __restrict__ nonfinite) {
  bool bad = false;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float v = g[i];
    bad |= !isfinite(v);
    g[i] = v * inv_scale;
  }
  if (bad) nonfinite[0] = 1;
}

__global__ void tanh_fwd_kernel(const float* __restrict__ x, long long n, float* __restrict__ y) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    y[i] = tanhf(x[i]);
}

__global__ void tanh_bwd_kernel(const float* __restrict__ y, const float* __restrict__ gy, long long n,
                                float* __restrict__ gx, int acc) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float t = y[i];
    const float g = gy[i] * (1.f - t * t);
    gx[i] = acc ? gx[i] + g : g;
  }
}

}  // namespace

extern "C" int dg_dmap_adaptive(const float* points, const int64_t* offsets, int N, int H, int W, double* sigma_ws,
                                float* dmap, void* stream) {
  DG_REQUIRE(offsets && dmap && sigma_ws && N > 0 && H > 0 && W > 0);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(dmap, 0, (size_t)N * H * W * 4, st) != hipSuccess) return DG_ERR_HIP;
  if (!points) return DG_OK;
  hipLaunchKernelGGL(knn_sigma_kernel, dim3(256), dim3(NT), 0, st, points, offsets, N, sigma_ws);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(dmap_adaptive_kernel, dim3(2048), dim3(NT), 0, st, points, offsets, N, H, W,
                     (const double*)sigma_ws, dmap);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_head_fwd(int dtype, const void* x, int64_t ldx, int M, int C, const float* w, const float* bias,
                           int act, float* y, void* stream) {
  DG_REQUIRE(x && w && y && M > 0 && C > 0 && act >= 0 && act <= 2);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(C % V == 0 && ldx % V == 0);
  hipStream_t st = (hipStream_t)stream;
  const int tpp_need = C / V;
  const int grid = ew_grid((long long)M * 16, 16384);
#define HF(T, TPP) hipLaunchKernelGGL((head_fwd_kernel<T, TPP>), dim3(grid), dim3(NT), 0, st, (const T*)x, ldx, M, C, w, bias, act, y)
  if (dtype == DG_BF16) {
    if (tpp_need >= 32) HF(bf16, 32); else if (tpp_need >= 16) HF(bf16, 16); else HF(bf16, 8);
  } else if (dtype == DG_F16) {
    if (tpp_need >= 32) HF(f16, 32); else if (tpp_need >= 16) HF(f16, 16); else HF(f16, 8);
  } else {
    if (tpp_need >= 32) HF(float, 32); else if (tpp_need >= 16) HF(float, 16); else HF(float, 8);
  }
#undef HF
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int64_t dg_head_workspace(int M, int C) {
  if (M <= 0 || C <= 0) return DG_ERR_INVALID;
  return (int64_t)head_nblk(M) * (C + 1) * 4;
}

extern "C" int dg_head_bwd(int dtype, const void* x, int64_t ldx, int M, int C, const float* w, int act,
                           const float* y, const float* gy, void* gx, int64_t ldgx, int accumulate_gx, float* gw,
                           float* gbias, void* workspace, void* stream) {
  DG_REQUIRE(x && w && y && gy && gw && workspace && M > 0 && C > 0 && act >= 0 && act <= 2);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  const int V = DG_IS16(dtype) ? 8 : 4;
  DG_SUPPORTED(C % V == 0 && C / V <= NT && ldx % V == 0 && (!gx || ldgx % V == 0));
  hipStream_t st = (hipStream_t)stream;
  const int nblk = head_nblk(M), ppb = dg_cdiv(M, nblk);
  float* part = (float*)workspace;
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(head_bwd_kernel<bf16>, dim3(nblk), dim3(NT), 0, st, (const bf16*)x, ldx, M, C, w, act, y, gy,
                       (bf16*)gx, ldgx, accumulate_gx, ppb, part);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(head_bwd_kernel<f16>, dim3(nblk), dim3(NT), 0, st, (const f16*)x, ldx, M, C, w, act, y, gy,
                       (f16*)gx, ldgx, accumulate_gx, ppb, part);
  else
    hipLaunchKernelGGL(head_bwd_kernel<float>, dim3(nblk), dim3(NT), 0, st, (const float*)x, ldx, M, C, w, act, y, gy,
                       (float*)gx, ldgx, accumulate_gx, ppb, part);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(colsum_kernel, dim3(C + 1), dim3(NT), 0, st, part, nblk, C + 1, gw, C, gbias);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int64_t dg_reduce_workspace(int64_t n) {
  if (n <= 0) return DG_ERR_INVALID;
  return (int64_t)ew_grid(n, 1024) * 4;
}

extern "C" int dg_mse_loss(const float* pred, const float* gt, float gt_scale, int64_t n, float* loss, float* dpred,
                           float grad_coef, void* workspace, void* stream) {
  DG_REQUIRE(pred && gt && loss && workspace && n > 0);
  hipStream_t st = (hipStream_t)stream;
  const int nblk = ew_grid(n, 1024);
  hipLaunchKernelGGL(mse_partial, dim3(nblk), dim3(NT), 0, st, pred, gt, gt_scale, (long long)n, dpred, grad_coef,
                     (float*)workspace);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(mse_final, dim3(1), dim3(64), 0, st, (const float*)workspace, nblk, (long long)n, loss);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_bce_loss(const float* pred, const float* target, int64_t n, float* loss, float* dpred,
                           float grad_coef, void* workspace, void* stream) {
  DG_REQUIRE(pred && target && loss && workspace && n > 0);
  hipStream_t st = (hipStream_t)stream;
  const int nblk = ew_grid(n, 1024);
  hipLaunchKernelGGL(bce_partial, dim3(nblk), dim3(NT), 0, st, pred, target, (long long)n, dpred, grad_coef,
                     (float*)workspace);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(mse_final, dim3(1), dim3(64), 0, st, (const float*)workspace, nblk, (long long)n, loss);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_adamw_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                             float beta2, float eps, float weight_decay, int step, void* stream) {
  DG_REQUIRE(p && g && m && v && n > 0 && step >= 1);
  const double bc1 = 1.0 - pow((double)beta1, step);
  const double bc2 = 1.0 - pow((double)beta2, step);
  const float step_size = (float)(lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  hipLaunchKernelGGL(adamw_kernel, dim3(ew_grid(n, 16384)), dim3(NT), 0, (hipStream_t)stream, p, g, m, v,
                     (long long)n, lr, beta1, beta2, eps, weight_decay, step_size, bc2_sqrt);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_gather_flat(const float* const* ptrs, const int64_t* offsets, int count, int64_t total,
                              float* flat, void* stream) {
  DG_REQUIRE(ptrs && offsets && flat && count > 0 && total > 0);
  // blocks over the whole buffer (the offsets are device-resident); chunks outside this run exit at once
  hipLaunchKernelGGL(gather_flat_kernel, dim3((unsigned)dg_cdiv(total, (int64_t)GATHER_CHUNK)), dim3(NT), 0,
                     (hipStream_t)stream, ptrs, offsets, count, flat);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_dmap_fixed(const float* points, const int64_t* offsets, int N, int H, int W, float sigma,
                             int radius, float* dmap, void* stream) {
  DG_REQUIRE(offsets && dmap && N > 0 && H > 0 && W > 0 && sigma > 0 && radius >= 0 && radius < 32);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(dmap, 0, (size_t)N * H * W * 4, st) != hipSuccess) return DG_ERR_HIP;
  if (!points) return DG_OK;
  hipLaunchKernelGGL(dmap_fixed_kernel, dim3(1024), dim3(NT), 0, st, points, offsets, N, H, W, sigma, radius, dmap);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_tanh_fwd(const float* x, int64_t n, float* y, void* stream) {
  DG_REQUIRE(x && y && n > 0);
  const int grid = (int)std::min<long long>(16384, (n + 255) / 256);
  hipLaunchKernelGGL(tanh_fwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, (long long)n, y);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_tanh_bwd(const float* y, const float* gy, int64_t n, float* gx, int accumulate, void* stream) {
  DG_REQUIRE(y && gy && gx && n > 0);
  const int grid = (int)std::min<long long>(16384, (n + 255) / 256);
  hipLaunchKernelGGL(tanh_bwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, y, gy, (long long)n, gx,
                     accumulate);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// no workspace (kept in the ABI for callers that size one: 0 bytes)
extern "C" int64_t dg_dmap_fixed_tiled_workspace(int N, int H, int W, int radius, int64_t npoints) {
  if (N <= 0 || H <= 0 || W <= 0 || radius < 0 || radius >= 32 || npoints < 0) return DG_ERR_INVALID;
  return 0;
}

extern "C" int dg_dmap_fixed_tiled(const float* points, const int64_t* offsets, int N, int H, int W, float sigma,
                                   int radius, int64_t npoints, void* workspace, float* dmap, void* stream) {
  (void)workspace;
  DG_REQUIRE(offsets && dmap && N > 0 && H > 0 && W > 0 && sigma > 0 && radius >= 0 && radius < 32);
  DG_REQUIRE(npoints >= 0 && (npoints == 0 || points));
  // DGVCC_DMAP_TILE (A/B): "64" (default), "64p", "32", "32p" -- tile rows, p = prefetched first chunk
  const char* e = getenv("DGVCC_DMAP_TILE");
  const bool wide = e && e[0] == 'w';  // "w": 16 x 256 tiles (1-KB row segments per wave store)
  const int rows = wide ? 16 : (e && e[0] == '3') ? 32 : 64, cols = wide ? 256 : 64;
  const bool pf = e && e[1] && e[2] == 'p';
  const int64_t T = (int64_t)((H + rows - 1) / rows) * ((W + cols - 1) / cols);
  DG_REQUIRE(T < (1ll << 31) && N < 65536);
  const dim3 grid((unsigned)T, (unsigned)N);
  hipStream_t st = (hipStream_t)stream;
  // the weights on the host (dmap_fixed_fused_kernel HOSTW; DGVCC_DMAP_HOSTW=0: formed per block)
  DmapWeights hw{};
  {
    const int K = 2 * radius + 1;
    double ex[64], sum = 0.0;
    for (int t = 0; t < K; ++t) {
      const int i = t - radius;
      ex[t] = std::exp(-0.5 / ((double)sigma * sigma) * (double)(i * i));
    }
    for (int j = 0; j < K; ++j) sum += ex[j];
    for (int t = 0; t < K; ++t) {
      hw.wd[t] = ex[t] / sum;
      hw.wf[t] = (float)hw.wd[t];
    }
  }
  const char* eh = getenv("DGVCC_DMAP_HOSTW");
  const bool hostw = !(eh && eh[0] == '0');
  // DGVCC_DMAP_PTS=1: chunks of 256 points (one per thread) instead of 512 (read per launch: A/B)
  const char* ec = getenv("DGVCC_DMAP_PTS");
  const bool pts2 = !(ec && ec[0] == '1');
  // DGVCC_DMAP_PERS=1: the tile-walking grid (measured slower: 22.4 vs 16.5 us on the bench's 16 frames);
  // default one block per (tile, image)
  const char* ep = getenv("DGVCC_DMAP_PERS");
  if (!e && ep && ep[0] == '1') {
    const long long tot = T * N;
    const unsigned g = (unsigned)std::min<long long>(tot, DMAP_PERS_BLOCKS);
    hipLaunchKernelGGL((dmap_fixed_fused_kernel<64, 0, 64, 1>), dim3(g), dim3(256), 0, st, points, offsets, H, W, sigma,
                       radius, dmap, N, hw);
    DG_CHECK_LAUNCH();
    return DG_OK;
  }
  if (wide) hipLaunchKernelGGL((dmap_fixed_fused_kernel<16, 0, 256>), grid, dim3(256), 0, st, points, offsets, H, W, sigma, radius, dmap, 1, hw);
  else if (rows == 32 && pf) hipLaunchKernelGGL((dmap_fixed_fused_kernel<32, 1>), grid, dim3(256), 0, st, points, offsets, H, W, sigma, radius, dmap, 1, hw);
  else if (rows == 32) hipLaunchKernelGGL((dmap_fixed_fused_kernel<32, 0>), grid, dim3(256), 0, st, points, offsets, H, W, sigma, radius, dmap, 1, hw);
  else if (pf) hipLaunchKernelGGL((dmap_fixed_fused_kernel<64, 1>), grid, dim3(256), 0, st, points, offsets, H, W, sigma, radius, dmap, 1, hw);
  else if (hostw && pts2) hipLaunchKernelGGL((dmap_fixed_fused_kernel<64, 0, 64, 0, 1, 2>), grid, dim3(256), 0, st, points, offsets, H, W, sigma, radius, dmap, 1, hw);
  else if (hostw) hipLaunchKernelGGL((dmap_fixed_fused_kernel<64, 0, 64, 0, 1>), grid, dim3(256), 0, st, points, offsets, H, W, sigma, radius, dmap, 1, hw);
  else hipLaunchKernelGGL((dmap_fixed_fused_kernel<64, 0>), grid, dim3(256), 0, st, points, offsets, H, W, sigma, radius, dmap, 1, hw);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_grad_unscale(float* g, int64_t n, float inv_scale, int* nonfinite, void* stream) {
  DG_REQUIRE(g && nonfinite && n > 0);
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(nonfinite, 0, sizeof(int), st) != hipSuccess) return DG_ERR_HIP;
  const int grid = (int)std::min<long long>(8192, (n + 255) / 256);
  hipLaunchKernelGGL(grad_unscale_kernel, dim3(grid), dim3(256), 0, st, g, (long long)n, inv_scale, nonfinite);
  DG_CHECK_LAUNCH();
  return DG_OK;
}
