// Bayesian loss (reference losses/bl.py): Post_Prob (:5-52) + Bay_Loss (:54-80).
//
// Per image b with n points and a G x G grid (G = c_size / stride, cell centres
// cood = k*stride + stride/2):
//   dis[i][j]  = (-2*y*cy + y*y + cy*cy) + (-2*x*cx + x*x + cx*cx)     (bl.py:27-31)
//   background (use_bg): dis[n][j] = (st_size*bg_ratio - sqrt(max(min_i dis[i][j], 0)))^2
//   prob[:, j] = softmax_i(-dis[:, j] / (2 sigma^2))                     (bl.py:44-45)
//   pre_count[i] = sum_j density[j] * prob[i][j]
//   res = |target - pre_count| (target of the background row = 0)
//   loss_b = sum of the ceil(0.9*(len(res)-1)) smallest res[:-1] + res[-1]   (bl.py:75-78)
//   loss = mean_b loss_b ; images without points: loss_b = |sum(density)|.
// The [n+1, G^2] posterior is never materialised: per-cell (max, sum) of the
// softmax is kept and the exponentials are recomputed in each pass.
#include "dg_common.h"
#include <algorithm>

namespace {

constexpr int NT = 256;

struct BLArgs {
  const float* pts;        // [total][2] (x, y)
  const int64_t* offs;     // [B+1]
  const float* st_sizes;   // [B]
  const float* targets;    // [total]
  const float* dens;       // [B][G*G]
  int B, G, use_bg;
  float stride, sigma, bg_ratio;
  float* cell;             // [B][G*G][3]: max logit, sum exp, bg logit
  float* count;            // [total + B]  pre_count (point rows, then one bg row per image)
  float* w;                // [total + B]  d loss_b / d pre_count
  float* img_loss;         // [B]
};

__device__ __forceinline__ float axis_dis(float p, float c) {
  float t = -2.f * (p * c);
  t = t + p * p;
  return t + c * c;
}

__device__ __forceinline__ float logit_of(const BLArgs& a, float x, float y, int j) {
  const int gy = j / a.G, gx = j - gy * a.G;
  const float cy = gy * a.stride + a.stride * 0.5f, cx = gx * a.stride + a.stride * 0.5f;
  const float d = axis_dis(y, cy) + axis_dis(x, cx);
  return -d / (2.f * a.sigma * a.sigma);
}

// pass 1: per cell softmax statistics over the image's points (+ background)
__global__ __launch_bounds__(NT) void bl_cells(BLArgs a) {
  const int b = blockIdx.y;
  const int G2 = a.G * a.G;
  const int j = blockIdx.x * NT + threadIdx.x;
  if (j >= G2) return;
  const int64_t p0 = a.offs[b], p1 = a.offs[b + 1];
  float* out = a.cell + ((long long)b * G2 + j) * 3;
  if (p1 == p0) { out[0] = 0.f; out[1] = 0.f; out[2] = 0.f; return; }
  float m = -INFINITY;
  for (int64_t i = p0; i < p1; ++i) m = fmaxf(m, logit_of(a, a.pts[2 * i], a.pts[2 * i + 1], j));
  float lbg = -INFINITY;
  if (a.use_bg) {
    // recompute the min distance exactly as the reference (min over dis)
    float md = INFINITY;
    const int gy = j / a.G, gx = j - gy * a.G;
    const float cy = gy * a.stride + a.stride * 0.5f, cx = gx * a.stride + a.stride * 0.5f;
    for (int64_t i = p0; i < p1; ++i) md = fminf(md, axis_dis(a.pts[2 * i + 1], cy) + axis_dis(a.pts[2 * i], cx));
    md = fmaxf(md, 0.f);
    const float dbg = a.st_sizes[b] * a.bg_ratio;
    const float t = dbg - sqrtf(md);
    lbg = -(t * t) / (2.f * a.sigma * a.sigma);
    m = fmaxf(m, lbg);
  }
  float s = 0.f;
  for (int64_t i = p0; i < p1; ++i) s += expf(logit_of(a, a.pts[2 * i], a.pts[2 * i + 1], j) - m);
  if (a.use_bg) s += expf(lbg - m);
  out[0] = m; out[1] = s; out[2] = lbg;
}

// pass 2: pre_count of every (point | background) row: one block per row
__global__ __launch_bounds__(NT) void bl_counts(BLArgs a, int total) {
  const int row = blockIdx.x;  // [0, total) points, [total, total + B) background rows
  const int G2 = a.G * a.G;
  int b;
  float x = 0.f, y = 0.f;
  bool bg = row >= total;
  if (bg) {
    b = row - total;
    if (!a.use_bg) return;
  } else {
    int lo = 0, hi = a.B;
    while (hi - lo > 1) { const int mid = (lo + hi) >> 1; if (a.offs[mid] <= row) lo = mid; else hi = mid; }
    b = lo;
    x = a.pts[2 * row]; y = a.pts[2 * row + 1];
  }
  const float* cell = a.cell + (long long)b * G2 * 3;
  const float* den = a.dens + (long long)b * G2;
  float s = 0.f;
  for (int j = threadIdx.x; j < G2; j += NT) {
    const float lg = bg ? cell[3 * j + 2] : logit_of(a, x, y, j);
    s += den[j] * (expf(lg - cell[3 * j]) / cell[3 * j + 1]);
  }
  s = wave_sum(s);
  __shared__ float sh[NT / 64];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) a.count[row] = sh[0] + sh[1] + sh[2] + sh[3];
}

// pass 3: per image residuals, trimmed sum (rank selection), d loss / d count
__global__ __launch_bounds__(NT) void bl_image_loss(BLArgs a, int total) {
  const int b = blockIdx.x;
  const int G2 = a.G * a.G;
  const int64_t p0 = a.offs[b], p1 = a.offs[b + 1];
  const int n = (int)(p1 - p0);
  __shared__ float red[NT];
  if (n == 0) {  // pre_count = sum(density), target 0, res = |sum|
    float s = 0.f;
    for (int j = threadIdx.x; j < G2; j += NT) s += a.dens[(long long)b * G2 + j];
    red[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
      for (int k = 0; k < NT; ++k) t += red[k];
      a.img_loss[b] = fabsf(t);
      a.w[total + b] = (t > 0.f) ? 1.f : (t < 0.f ? -1.f : 0.f);  // flag: whole-map gradient
    }
    return;
  }
  // rows of res: n points (+ background as the last one when use_bg)
  const int L = a.use_bg ? n + 1 : n;
  auto res_of = [&](int k) -> float {
    if (k < n) {
      const float tg = a.targets[p0 + k];
      return fabsf(tg - a.count[p0 + k]);
    }
    return fabsf(0.f - a.count[total + b]);
  };
  const int num = (int)ceil(0.9 * (double)(L - 1));  // Python float math: ceil(0.9 * (len(res) - 1))
  float acc = 0.f;
  for (int k = threadIdx.x; k < L - 1; k += NT) {
    const float rk = res_of(k);
    int rank = 0;
    for (int q = 0; q < L - 1; ++q) {
      const float rq = res_of(q);
      rank += (rq < rk) || (rq == rk && q < k);
    }
    const bool sel = rank < num;
    const float cnt = k < n ? a.count[p0 + k] : a.count[total + b];
    const float tg = k < n ? a.targets[p0 + k] : 0.f;
    const float sgn = (cnt > tg) ? 1.f : (cnt < tg ? -1.f : 0.f);
    if (sel) acc += rk;
    const float wv = sel ? sgn : 0.f;
    if (k < n) a.w[p0 + k] = wv; else a.w[total + b] = wv;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < NT; ++k) t += red[k];
    // the last row always counts
    const int k = L - 1;
    const float rk = res_of(k);
    const float cnt = k < n ? a.count[p0 + k] : a.count[total + b];
    const float tg = k < n ? a.targets[p0 + k] : 0.f;
    const float sgn = (cnt > tg) ? 1.f : (cnt < tg ? -1.f : 0.f);
    if (k < n) a.w[p0 + k] = sgn; else a.w[total + b] = sgn;
    a.img_loss[b] = t + rk;
  }
}

__global__ void bl_mean(const float* img_loss, int B, float* loss) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    float t = 0.f;
    for (int b = 0; b < B; ++b) t += img_loss[b];
    loss[0] = t / (float)B;
  }
}

// pass 4: d loss / d density[b][j] = coef/B * sum_rows w_row * prob[row][j]
__global__ __launch_bounds__(NT) void bl_grad(BLArgs a, int total, const float* coef, float* gd) {
  const int b = blockIdx.y;
  const int G2 = a.G * a.G;
  const int j = blockIdx.x * NT + threadIdx.x;
  if (j >= G2) return;
  const float k = (coef ? coef[0] : 1.f) / (float)a.B;
  const int64_t p0 = a.offs[b], p1 = a.offs[b + 1];
  if (p1 == p0) {
    gd[(long long)b * G2 + j] = k * a.w[total + b];
    return;
  }
  const float* cell = a.cell + ((long long)b * G2 + j) * 3;
  const float m = cell[0], rs = 1.f / cell[1];
  float g = 0.f;
  for (int64_t i = p0; i < p1; ++i) {
    const float wi = a.w[i];
    if (wi != 0.f) g += wi * (expf(logit_of(a, a.pts[2 * i], a.pts[2 * i + 1], j) - m) * rs);
  }
  if (a.use_bg) g += a.w[total + b] * (expf(cell[2] - m) * rs);
  gd[(long long)b * G2 + j] = k * g;
}

// Post_Prob materialised: prob rows of image b at out + rowoff[b] * G2
__global__ __launch_bounds__(NT) void bl_prob(BLArgs a, const int64_t* rowoff, float* out) {
  const int b = blockIdx.y;
  const int G2 = a.G * a.G;
  const int j = blockIdx.x * NT + threadIdx.x;
  if (j >= G2) return;
  const int64_t p0 = a.offs[b], p1 = a.offs[b + 1];
  const float* cell = a.cell + ((long long)b * G2 + j) * 3;
  const float m = cell[0], rs = 1.f / cell[1];
  float* o = out + rowoff[b] * G2 + j;
  for (int64_t i = p0; i < p1; ++i)
    o[(i - p0) * G2] = expf(logit_of(a, a.pts[2 * i], a.pts[2 * i + 1], j) - m) * rs;
  if (a.use_bg && p1 > p0) o[(p1 - p0) * G2] = expf(cell[2] - m) * rs;
}

}  // namespace

extern "C" int dg_bl_prob(const float* points, const int64_t* offsets, int64_t total_points, const float* st_sizes,
                          int B, int G, float stride, float sigma, float bg_ratio, int use_bg,
                          const int64_t* row_offsets, float* prob, void* workspace, void* stream) {
  DG_REQUIRE(offsets && st_sizes && row_offsets && prob && workspace && B > 0 && G > 0 && sigma > 0);
  DG_REQUIRE(total_points == 0 || points);
  hipStream_t st = (hipStream_t)stream;
  BLArgs a{};
  a.pts = points; a.offs = offsets; a.st_sizes = st_sizes;
  a.B = B; a.G = G; a.use_bg = use_bg; a.stride = stride; a.sigma = sigma; a.bg_ratio = bg_ratio;
  a.cell = (float*)workspace;
  const int G2 = G * G;
  hipLaunchKernelGGL(bl_cells, dim3(dg_cdiv(G2, NT), B), dim3(NT), 0, st, a);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(bl_prob, dim3(dg_cdiv(G2, NT), B), dim3(NT), 0, st, a, row_offsets, prob);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int64_t dg_bl_workspace(int B, int G, int64_t total_points) {
  if (B <= 0 || G <= 0 || total_points < 0) return DG_ERR_INVALID;
  return ((int64_t)B * G * G * 3 + 2 * (total_points + B) + B) * 4;
}

extern "C" int dg_bl_loss(const float* points, const int64_t* offsets, int64_t total_points, const float* st_sizes,
                          const float* targets, const float* density, int B, int G, float stride, float sigma,
                          float bg_ratio, int use_bg, float* loss, float* ddensity, const float* grad_coef,
                          void* workspace, void* stream) {
  DG_REQUIRE(offsets && st_sizes && density && loss && workspace && B > 0 && G > 0 && sigma > 0 && stride > 0);
  DG_REQUIRE(total_points == 0 || (points && targets));
  DG_SUPPORTED(total_points < (1ll << 31));
  hipStream_t st = (hipStream_t)stream;
  float* ws = (float*)workspace;
  BLArgs a;
  a.pts = points; a.offs = offsets; a.st_sizes = st_sizes; a.targets = targets; a.dens = density;
  a.B = B; a.G = G; a.use_bg = use_bg; a.stride = stride; a.sigma = sigma; a.bg_ratio = bg_ratio;
  a.cell = ws;
  a.count = ws + (long long)B * G * G * 3;
  a.w = a.count + total_points + B;
  a.img_loss = a.w + total_points + B;
  const int total = (int)total_points;
  const int G2 = G * G;
  hipLaunchKernelGGL(bl_cells, dim3(dg_cdiv(G2, NT), B), dim3(NT), 0, st, a);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(bl_counts, dim3(total + B), dim3(NT), 0, st, a, total);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(bl_image_loss, dim3(B), dim3(NT), 0, st, a, total);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(bl_mean, dim3(1), dim3(64), 0, st, (const float*)a.img_loss, B, loss);
  DG_CHECK_LAUNCH();
  if (ddensity) {
    hipLaunchKernelGGL(bl_grad, dim3(dg_cdiv(G2, NT), B), dim3(NT), 0, st, a, total, grad_coef, ddensity);
    DG_CHECK_LAUNCH();
  }
  return DG_OK;
}
