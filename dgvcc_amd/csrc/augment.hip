// Device-side training augmentation of DenClsDataset:
//   datasets/den_cls_dataset.py:77-158 (_train_transform: grey, hflip, ToTensor +
//   Normalize -> view 1) and :29-35 (more_transform: RandomApply(ColorJitter(0.5, 0.2,
//   0.2, 0.1), p=.8), RandomApply(GaussianBlur(3, 1), p=.5), RandomAdjustSharpness(5, p=.5),
//   ToTensor + Normalize -> view 2), and the block map of :62-63.
//
// The reference runs these on PIL images on host worker processes.  Here every sample
// of a batch is a uint8 HWC crop already resident in HBM; the random decisions are
// drawn on the host in the reference's RNG order (dgvcc_amd/datasets) and passed as
// per-sample parameters.  Every PIL step keeps PIL's integer semantics so the result is
// bit-identical to the reference's host pipeline:
//   * convert('L'):   L = (19595 R + 38470 G + 7471 B + 0x8000) >> 16
//   * Image.blend:    out = clip(trunc(in1 + a * (in2 - in1))) in float32
//                     (ImageEnhance Brightness / Contrast / Color / Sharpness)
//   * Contrast mean:  int(mean(L) + 0.5)
//   * RGB<->HSV:      PIL's float/double mix (exhaustively checked over all 2^24 inputs)
//   * SMOOTH filter:  3x3 [1 1 1; 1 5 1; 1 1 1] / 13, round half up, border pixels kept
//   * GaussianBlur:   torchvision's tensor path (float32 separable-weight 3x3 conv,
//                     reflect padding, round half to even)
// Byte-wise HBM passes (one per applied op); per-image reductions for the contrast mean.
#include "dg_common.h"
#include <algorithm>

// PIL's C code and torchvision's CPU arithmetic are not contracted into FMAs: keep every
// multiply-add of this file as two roundings (except the explicit fmaf of the blur).
#pragma clang fp contract(off)

namespace {

constexpr int NT = 256;

// per-sample parameter record (host: dgvcc_amd/datasets/augment.py AUG_PARAMS)
// P_HUE_SHIFT: uint8(hue_factor * 255) as numpy computes it (host); P_K0/P_K1: the
// torchvision 1-D Gaussian weights (edge, centre), computed on the host in float32 exactly
// as _get_gaussian_kernel1d does.
enum {
  P_GREY = 0, P_FLIP, P_JITTER, P_ORDER0, P_ORDER1, P_ORDER2, P_ORDER3, P_BRIGHT, P_CONTRAST, P_SAT, P_HUE_SHIFT,
  P_BLUR, P_K0, P_K1, P_SHARP, P_SHARP_F, P_COUNT
};
static_assert(P_COUNT == 16, "parameter record");
constexpr int PSTRIDE = 16;

__device__ __forceinline__ int lum(int r, int g, int b) { return (19595 * r + 38470 * g + 7471 * b + 0x8000) >> 16; }

__device__ __forceinline__ int blend8(float in1, float in2, float a) {
  const float t = in1 + a * (in2 - in1);
  return t <= 0.f ? 0 : (t >= 255.f ? 255 : (int)t);
}

__device__ __forceinline__ float norm_px(int v) {  // ToTensor (x / 255) + Normalize(0.5, 0.5)
  const float t = (float)v / 255.f;
  return (t - 0.5f) / 0.5f;
}

// PIL rgb2hsv_row
__device__ __forceinline__ void rgb2hsv(int r, int g, int b, int& uh, int& us, int& uv) {
  const int maxc = max(r, max(g, b)), minc = min(r, min(g, b));
  uv = maxc;
  if (minc == maxc) { uh = 0; us = 0; return; }
  const float cr = (float)(maxc - minc);
  const float s = cr / (float)maxc;
  const float rc = (float)(maxc - r) / cr, gc = (float)(maxc - g) / cr, bc = (float)(maxc - b) / cr;
  float h;
  if (r == maxc) h = bc - gc;
  else if (g == maxc) h = (float)(2.0 + (double)rc - (double)bc);
  else h = (float)(4.0 + (double)gc - (double)rc);
  h = (float)fmod((double)h / 6.0 + 1.0, 1.0);
  uh = min(255, max(0, (int)((double)h * 255.0)));
  us = min(255, max(0, (int)((double)s * 255.0)));
}

// PIL hsv2rgb
__device__ __forceinline__ void hsv2rgb(int h, int s, int v, int& r, int& g, int& b) {
  if (s == 0) { r = g = b = v; return; }
  const double hf = (double)h * 6.0 / 255.0;
  const int i = (int)floor(hf);
  const double f = hf - (double)i;
  const double fs = (double)s / 255.0;
  const int p = min(255, max(0, (int)rint((double)v * (1.0 - fs))));
  const int q = min(255, max(0, (int)rint((double)v * (1.0 - fs * f))));
  const int t = min(255, max(0, (int)rint((double)v * (1.0 - fs * (1.0 - f)))));
  switch (i % 6) {
    case 0: r = v; g = t; b = p; break;
    case 1: r = q; g = v; b = p; break;
    case 2: r = p; g = v; b = t; break;
    case 3: r = p; g = q; b = v; break;
    case 4: r = t; g = p; b = v; break;
    default: r = v; g = p; b = q; break;
  }
}

// view 1 and the base image of view 2: grey (convert('L').convert('RGB')), hflip,
// then ToTensor + Normalize into img1 (NCHW f32).  One thread per pixel.
__global__ __launch_bounds__(NT) void aug_base_kernel(const unsigned char* __restrict__ in, int B, int H, int W,
                                                      const float* __restrict__ prm, unsigned char* __restrict__ base,
                                                      float* __restrict__ img1) {
  const long long HW = (long long)H * W;
  const long long total = B * HW;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int n = (int)(i / HW);
    const int rem = (int)(i - n * HW);
    const int y = rem / W, x = rem - y * W;
    const float* p = prm + n * PSTRIDE;
    const int xs = p[P_FLIP] != 0.f ? W - 1 - x : x;  // F.hflip
    const unsigned char* s = in + (((long long)n * H + y) * W + xs) * 3;
    int r = s[0], g = s[1], b = s[2];
    if (p[P_GREY] != 0.f) r = g = b = lum(r, g, b);
    unsigned char* d = base + i * 3;
    d[0] = (unsigned char)r; d[1] = (unsigned char)g; d[2] = (unsigned char)b;
    float* o = img1 + (long long)n * 3 * HW + rem;
    o[0] = norm_px(r); o[HW] = norm_px(g); o[2 * HW] = norm_px(b);
  }
}

// ImageStat sum of convert('L') per image: exact integer partial sums of 64 blocks per image,
// combined with integer atomics (order-independent, so deterministic).
constexpr int LM_BLOCKS = 64;
__global__ __launch_bounds__(NT) void aug_lsum_kernel(const unsigned char* __restrict__ img, int H, int W,
                                                      unsigned long long* __restrict__ lsum) {
  __shared__ unsigned long long sh[NT];
  const long long HW = (long long)H * W;
  const int n = blockIdx.y;
  const unsigned char* s = img + n * HW * 3;
  unsigned long long acc = 0;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < HW; i += (long long)LM_BLOCKS * NT)
    acc += (unsigned)lum(s[i * 3], s[i * 3 + 1], s[i * 3 + 2]);
  sh[threadIdx.x] = acc;
  __syncthreads();
  for (int o = NT / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicAdd(lsum + n, sh[0]);
}

// One ColorJitter round: sample n applies op order[k] (0 brightness, 1 contrast,
// 2 saturation, 3 hue) with torchvision's PIL implementations; samples without the
// jitter copy through.
__global__ __launch_bounds__(NT) void aug_jitter_kernel(const unsigned char* __restrict__ in, int B, int H, int W,
                                                        const float* __restrict__ prm, int k,
                                                        const unsigned long long* __restrict__ lsum,
                                                        unsigned char* __restrict__ out) {
  const long long HW = (long long)H * W;
  const long long total = B * HW;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int n = (int)(i / HW);
    const float* p = prm + n * PSTRIDE;
    const unsigned char* s = in + i * 3;
    int r = s[0], g = s[1], b = s[2];
    if (p[P_JITTER] != 0.f) {
      const int op = (int)p[P_ORDER0 + k];
      if (op == 0) {
        const float a = p[P_BRIGHT];
        r = blend8(0.f, (float)r, a); g = blend8(0.f, (float)g, a); b = blend8(0.f, (float)b, a);
      } else if (op == 1) {
        // ImageEnhance.Contrast: int(ImageStat mean of L + 0.5)
        const float a = p[P_CONTRAST], m = (float)(int)((double)lsum[n] / (double)HW + 0.5);
        r = blend8(m, (float)r, a); g = blend8(m, (float)g, a); b = blend8(m, (float)b, a);
      } else if (op == 2) {
        const float a = p[P_SAT], l = (float)lum(r, g, b);
        r = blend8(l, (float)r, a); g = blend8(l, (float)g, a); b = blend8(l, (float)b, a);
      } else {
        // F_pil.adjust_hue: uint8 H channel += uint8(hue_factor * 255), wrapping
        int hh, ss, vv;
        rgb2hsv(r, g, b, hh, ss, vv);
        hh = (hh + (int)p[P_HUE_SHIFT]) & 255;
        hsv2rgb(hh, ss, vv, r, g, b);
      }
    }
    unsigned char* d = out + i * 3;
    d[0] = (unsigned char)r; d[1] = (unsigned char)g; d[2] = (unsigned char)b;
  }
}

__device__ __forceinline__ int reflect(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }

// GaussianBlur(3, sigma) on the uint8 image (torchvision F_t.gaussian_blur), then
// RandomAdjustSharpness(5) (PIL), then ToTensor + Normalize into img2.  The blur and the
// sharpness read neighbourhoods, so each is its own pass (stage 0: blur, 1: sharpness + normalise).
__global__ __launch_bounds__(NT) void aug_blur_kernel(const unsigned char* __restrict__ in, int B, int H, int W,
                                                      const float* __restrict__ prm, unsigned char* __restrict__ out) {
  const long long HW = (long long)H * W;
  const long long total = B * HW;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int n = (int)(i / HW);
    const int rem = (int)(i - n * HW);
    const int y = rem / W, x = rem - y * W;
    const float* p = prm + n * PSTRIDE;
    const unsigned char* img = in + (long long)n * HW * 3;
    unsigned char* d = out + i * 3;
    if (p[P_BLUR] == 0.f) {
      d[0] = img[rem * 3]; d[1] = img[rem * 3 + 1]; d[2] = img[rem * 3 + 2];
      continue;
    }
    // kernel2d = outer(k1d, k1d), k1d = (k0, k1, k0) (torchvision _get_gaussian_kernel2d)
    const float k1[3] = {p[P_K0], p[P_K1], p[P_K0]};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float acc = 0.f;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const int yy = reflect(y + dy - 1, H);
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const int xx = reflect(x + dx - 1, W);
          acc = fmaf(k1[dy] * k1[dx], (float)img[((long long)yy * W + xx) * 3 + c], acc);
        }
      }
      d[c] = (unsigned char)rintf(acc);  // torch.round (half to even), then .to(uint8)
    }
  }
}

__global__ __launch_bounds__(NT) void aug_sharp_norm_kernel(const unsigned char* __restrict__ in, int B, int H, int W,
                                                            const float* __restrict__ prm,
                                                            float* __restrict__ img2) {
  const long long HW = (long long)H * W;
  const long long total = B * HW;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int n = (int)(i / HW);
    const int rem = (int)(i - n * HW);
    const int y = rem / W, x = rem - y * W;
    const float* p = prm + n * PSTRIDE;
    const unsigned char* img = in + (long long)n * HW * 3;
    int v[3] = {img[rem * 3], img[rem * 3 + 1], img[rem * 3 + 2]};
    if (p[P_SHARP] != 0.f && y > 0 && y < H - 1 && x > 0 && x < W - 1) {  // PIL keeps the border pixels
      const float a = p[P_SHARP_F];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        int acc = 0;
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
          for (int dx = -1; dx <= 1; ++dx)
            acc += (dy == 0 && dx == 0 ? 5 : 1) * img[((long long)(y + dy) * W + x + dx) * 3 + c];
        const int sm = (2 * acc + 13) / 26;  // round half up of acc / 13
        v[c] = blend8((float)sm, (float)v[c], a);
      }
    }
    float* o = img2 + (long long)n * 3 * HW + rem;
    o[0] = norm_px(v[0]); o[HW] = norm_px(v[1]); o[2 * HW] = norm_px(v[2]);
  }
}

// bmap = (16x16 block sums of dmap > 0) (datasets/den_cls_dataset.py:62-63); one thread per block
// (the block sum in float32, row-major order as torch's reshape-sum on a contiguous tensor).
__global__ __launch_bounds__(NT) void aug_bmap_kernel(const float* __restrict__ dmap, int B, int h, int w,
                                                      float* __restrict__ bmap) {
  const int bh = h / 16, bw = w / 16;
  const long long total = (long long)B * bh * bw;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
    const int n = (int)(i / (bh * bw));
    const int rem = (int)(i - (long long)n * bh * bw);
    const int by = rem / bw, bx = rem - by * bw;
    float s = 0.f;
    for (int y = 0; y < 16; ++y)
      for (int x = 0; x < 16; ++x) s += dmap[((long long)n * h + by * 16 + y) * w + bx * 16 + x];
    bmap[i] = s > 0.f ? 1.f : 0.f;
  }
}

inline int ew_grid(long long n) { return (int)std::max<long long>(1, std::min<long long>((n + NT - 1) / NT, 16384)); }

}  // namespace

extern "C" int64_t dg_augment_workspace(int B, int H, int W) {
  if (B <= 0 || H <= 0 || W <= 0) return DG_ERR_INVALID;
  return 2 * (int64_t)B * H * W * 3 + 8 * (int64_t)B + 64;
}

extern "C" int dg_augment_den_cls(const unsigned char* imgs, int B, int H, int W, const float* params, float* img1,
                                  float* img2, void* workspace, int64_t ws_bytes, void* stream) {
  DG_REQUIRE(imgs && params && img1 && img2 && workspace && B > 0 && H >= 3 && W >= 3);
  DG_REQUIRE(ws_bytes >= dg_augment_workspace(B, H, W));
  DG_SUPPORTED((long long)B * H * W < (1LL << 31));
  hipStream_t st = (hipStream_t)stream;
  const long long npx = (long long)B * H * W;
  unsigned char* bufA = (unsigned char*)workspace;
  unsigned char* bufB = bufA + npx * 3;
  unsigned long long* lsum = (unsigned long long*)(((uintptr_t)(bufB + npx * 3) + 15) & ~(uintptr_t)15);
  const int g = ew_grid(npx);
  hipLaunchKernelGGL(aug_base_kernel, dim3(g), dim3(NT), 0, st, imgs, B, H, W, params, bufA, img1);
  DG_CHECK_LAUNCH();
  unsigned char* cur = bufA;
  unsigned char* nxt = bufB;
  for (int k = 0; k < 4; ++k) {  // ColorJitter rounds in each sample's permuted order
    if (hipMemsetAsync(lsum, 0, sizeof(unsigned long long) * B, st) != hipSuccess) return DG_ERR_HIP;
    hipLaunchKernelGGL(aug_lsum_kernel, dim3(LM_BLOCKS, B), dim3(NT), 0, st, cur, H, W, lsum);
    DG_CHECK_LAUNCH();
    hipLaunchKernelGGL(aug_jitter_kernel, dim3(g), dim3(NT), 0, st, cur, B, H, W, params, k, lsum, nxt);
    DG_CHECK_LAUNCH();
    std::swap(cur, nxt);
  }
  hipLaunchKernelGGL(aug_blur_kernel, dim3(g), dim3(NT), 0, st, cur, B, H, W, params, nxt);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(aug_sharp_norm_kernel, dim3(g), dim3(NT), 0, st, nxt, B, H, W, params, img2);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_block_map(const float* dmap, int B, int h, int w, float* bmap, void* stream) {
  DG_REQUIRE(dmap && bmap && B > 0 && h > 0 && w > 0);
  DG_SUPPORTED(h % 16 == 0 && w % 16 == 0);
  const long long n = (long long)B * (h / 16) * (w / 16);
  hipLaunchKernelGGL(aug_bmap_kernel, dim3(ew_grid(n)), dim3(NT), 0, (hipStream_t)stream, dmap, B, h, w, bmap);
  DG_CHECK_LAUNCH();
  return DG_OK;
}
