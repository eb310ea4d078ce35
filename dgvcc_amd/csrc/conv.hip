// Implicit-GEMM convolution for gfx950 (MI355X): forward, data-grad and
// weight-grad of the stride-1 "same" convolutions on the DGVCC hot path
// (vgg16_bn.features convs, models/models.py:35-38; ConvBlock
// models/models.py:8-21; cls_head models/models.py:238-243).
//
// GEMM view (NHWC activations, weights packed [Cout][R][S][C]):
//   forward  D[co][px] = sum_{r,s,c} W[co][r][s][c] * X[px + (r-pad, s-pad)][c]
//   wgrad    D[co][(r,s,c)] = sum_px dY[px][co] * X[px + (r-pad, s-pad)][c]
//   dgrad    = forward of dY with the flipped, transposed filter.
// Each K-tile row is 128 bytes (64 bf16 / 32 f32 channels of one (r,s) tap),
// staged global->registers->LDS (XOR-swizzled, double buffered, one barrier per
// K-tile) and consumed by v_mfma_f32_16x16x32_bf16 (perf mode) or the exact
// f32 v_mfma_f32_16x16x4_f32 (parity mode).  Out-of-image taps are zero-filled
// by the buffer-load range check (voffset past num_records returns 0).
#include <mutex>
#include "dg_common.h"
#include <algorithm>
#include <cstdlib>

namespace {

constexpr int NT = 256;  // 4 waves, 2x2 over the output tile

struct FwdArgs {
  const char* x; long long ldx; int N, H, W, C;
  const char* w; int Cout, R, S, pad;
  const float* bias;
  char* y; long long ldy;
  int accumulate;
  float* part = nullptr;   // bf16 pipe/tap3 only: BN statistics partials [ceil(M/256)][3][Cout]
  int ksplit = 1;          // bf16 pipe only: > 1 splits the K loop over blocks, f32 partials into kpart
  float* kpart = nullptr;  // [ksplit][M][Cout]; splitk_reduce_kernel finishes bias/accumulate/stats
  // bf16 pipe only, dgrad launches: the BatchNorm-backward partial sums of the layer whose
  // output gradient this launch produces (norm.hip bn_bwd_partial's three rows per
  // 256-pixel tile: sum g', sum g' xhat, sum xhat with g' = g * drop * relu'(bn(z)))
  const char* bz = nullptr;
  long long ldbz = 0;
  const float *bsc = nullptr, *bsf = nullptr, *bmu = nullptr, *bis = nullptr, *bdrop = nullptr;
  int bact = 0, bHW = 1;
  float* bpart = nullptr;
  // eval-mode BatchNorm (+ReLU) in the epilogue: y = act(conv*escale + eshift), applied after
  // bias/accumulate exactly as dg_bn_apply applies it to a stored f32 z
  const float* escale = nullptr;
  const float* eshift = nullptr;
  int eact = 0;
  int tile_order = 0;  // f32 pre-split kernel: 1 = channel-tile-major tile walk (DGVCC_PSPLIT_ORDER)
  // K-step order of the persistent / pre-split / 16-bit pipeline kernels: 0 = tap-major (kt = rs * CB + cb), 1 =
  // channel-block-major (kt = cb * RS + rs: the 9 taps of one channel block back to back, so a
  // tile's pixel window for that block is re-read from L2 by the next 8 taps instead of after all
  // CB blocks of the tap, when 32 tiles per XCD of windows no longer fit the 4-MB L2: on the
  // 512 -> 512 f32 layer HBM fetch 9.1 -> 2.7 GB per launch, L2 hit rate 85 -> 95%)
  int korder = 0;
  // f32 split math: caller-owned room for the pre-split filter planes (3 bf16 planes of the
  // Cout*R*S*C filter, dg_conv_fwd_workspace); null / too small: kernels that split per wave
  char* wsplit = nullptr;
  long long wsplit_bytes = 0;
  // dg_conv_fwd_acc_relu (accumulating 1x1 dgrad whose output is the gradient of a ReLU output):
  // the ReLU output, same dtype / rows as y; the accumulated value is zeroed where it is <= 0
  const char* rmask = nullptr;
  long long ldrm = 0;
  // 16-bit persistent / pipe forward: 16-byte epilogue stores (lane pairs exchange halves with
  // v_permlane16_swap); set by launch_fwd where y's rows are 16-byte aligned (DGVCC_PERS_WST)
  int wide_st = 0;
  // f32 f16 x3 arithmetic: a device float >= max |x| (NULL: presplit_h runs amax_kernel over x)
  const float* xamax = nullptr;
  // f32 f16 x3: x's pair image written by its producer (dg_bn_apply_pair, the SCH 8 layout) and the
  // bound its scale came from; the pre-split forward then reads it (no split_x_h pass, no in-kernel
  // split) with the bound as its xamax; other kernels use x and xamax
  const char* xpair = nullptr;
  const float* xbound = nullptr;
  // diagnostic stamp rows (conv_fwd_psplit_kernel STAMP = 1; dg_debug_stamps)
  unsigned long long* stamps = nullptr;
};
template <typename T> __device__ __forceinline__ unsigned pack2(float lo, float hi);
template <> __device__ __forceinline__ unsigned pack2<bf16>(float lo, float hi) { return pack_bf2(lo, hi); }
template <> __device__ __forceinline__ unsigned pack2<f16>(float lo, float hi) { return pack_h2(lo, hi); }

// EPI_ACC_NOTE -- conv epilogues: y += old y (accumulate) runs as a pass of its own ahead of the
// stores, acc = (acc + bias) + y_old with the loads issued together, and the store loop adds the
// bias only when not accumulating (the same float operations in the same order).  With the y load
// inside the store loop behind the runtime `accumulate` branch, the compiler drained vmcnt to 0 in
// front of every store, so each store waited for the previous ones (and for the next tile's DMA in
// the persistent kernels); the store loop now holds no global loads and its stores issue back to
// back.  (Bias values come from registers or LDS for the same reason.)
__device__ __forceinline__ void epi_affine(float v[4], const FwdArgs& a, int co) {
  if (!a.escale) return;
  const f4v sc = *(const f4v*)(a.escale + co), sf = *(const f4v*)(a.eshift + co);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float t = fmaf(v[r], sc[r], sf[r]);
    if (a.eact == 1) t = t > 0.f ? t : 0.f;
    v[r] = t;
  }
}

// y += old y of the accumulate prepass (EPI_ACC_NOTE).  With a.rmask the sum is zeroed where the
// ReLU output at (px, co) is <= 0 -- relu_bwd_kernel's rule, applied by the launch that produces
// the gradient instead of by a pass of its own over it (dg_conv_fwd_acc_relu)
template <typename T, typename V>
__device__ __forceinline__ void add_old_y(V& v, const T* yrow, const FwdArgs& a, long long px, int co) {
  float o[4];
  ld4(yrow + co, o);
  if (a.rmask) {
    float m[4];
    ld4((const T*)a.rmask + px * a.ldrm + co, m);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = m[r] > 0.f ? v[r] + o[r] : 0.f;
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += o[r];
  }
}

// Sum over the 16 lanes of a DPP row, result in every lane: quad butterflies (xor 1, 2)
// then rotations by 4 and 8 (VALU-only, no LDS crossbar traffic).
#define DG_DPP(x, ctrl) __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), (ctrl), 0xf, 0xf, true))
__device__ __forceinline__ float row16_sum(float x) {
  x += DG_DPP(x, 0xB1);   // quad_perm [1,0,3,2]
  x += DG_DPP(x, 0x4E);   // quad_perm [2,3,0,1]
  x += DG_DPP(x, 0x124);  // row_ror:4
  x += DG_DPP(x, 0x128);  // row_ror:8
  return x;
}

// Workgroup barrier for LDS hand-offs only: unlike __syncthreads() it does not wait for
// this wave's outstanding global stores (the epilogue's y stores keep draining).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Epilogue BN statistics of the stored (bf16-rounded) conv outputs, replacing the
// separate statistics pass over z (norm.hip bn_stats_partial).  acc holds the stored
// values; lane (fr, fc) has channels cw + 16i + 4fc + r of pixel 16j + fr of its wave.
// Per wave and channel: count, mean and M2 over its valid pixels (DPP row sums over
// the 16 pixel lanes, two passes over registers), then a Chan merge of the NPW pixel
// waves through LDS into one partial row (n, mean, M2) per block.
template <int TI, int TJ, int NPW, int BN>
__device__ __forceinline__ void epi_stats(f4v (&acc)[TI][TJ], const bool (&valid)[TJ], int pw, int cw, char* lds,
                                          float* part_row, int Cout, int co0, int tid, int fr, int fc) {
  float cnt = 0.f;
#pragma unroll
  for (int j = 0; j < TJ; ++j) cnt += valid[j] ? 1.f : 0.f;
  cnt = row16_sum(cnt);
  const float rcnt = cnt > 0.f ? 1.f / cnt : 0.f;
  float* sh = (float*)lds;  // [NPW][3][BN]
  lds_barrier();            // every wave is done reading the operand ring
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float sm = 0.f;
#pragma unroll
      for (int j = 0; j < TJ; ++j) sm += valid[j] ? acc[i][j][r] : 0.f;
      const float mean = row16_sum(sm) * rcnt;
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const float d = acc[i][j][r] - mean;
        q = valid[j] ? fmaf(d, d, q) : q;
      }
      q = row16_sum(q);
      if (fr == 0) {
        const int c = cw + 16 * i + 4 * fc + r;
        sh[(pw * 3 + 0) * BN + c] = cnt;
        sh[(pw * 3 + 1) * BN + c] = mean;
        sh[(pw * 3 + 2) * BN + c] = q;
      }
    }
  lds_barrier();
  for (int c = tid; c < BN; c += 64 * 4 * NPW) {
    float n = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
    for (int w = 0; w < NPW; ++w) {
      const float nb = sh[(w * 3 + 0) * BN + c];
      if (nb == 0.f) continue;
      const float mb = sh[(w * 3 + 1) * BN + c];
      const float nt = n + nb;
      const float d = mb - mean;
      mean += d * (nb / nt);
      m2 += sh[(w * 3 + 2) * BN + c] + d * d * (n * nb / nt);
      n = nt;
    }
    part_row[co0 + c] = n;
    part_row[Cout + co0 + c] = mean;
    part_row[2 * Cout + co0 + c] = m2;
  }
}

// Epilogue BatchNorm-backward partial sums of the stored (bf16-rounded) gradient tile:
// the separate pass over (g, z) of norm.hip's bn_bwd_partial, computed where g is
// produced; z is read here at the tile's pixels (8-B loads), once.
template <int TI, int TJ, int NPW, int BN, typename T = bf16, int PXT = 256>
__device__ __forceinline__ void epi_bnbwd(f4v (&acc)[TI][TJ], const bool (&valid)[TJ], int pw, int cw, int wpx,
                                          char* lds, const FwdArgs& a, int px0, int co0, int tid, int fr, int fc) {
  float* sh = (float*)lds;  // [NPW][3][BN]
  lds_barrier();            // every wave is done reading the operand ring
  const T* z = (const T*)a.bz;
#pragma unroll
  for (int i = 0; i < TI; ++i) {
    const int cl = cw + 16 * i + 4 * fc;
    const int c = co0 + cl;
    float sc[4], sf[4], mu[4], is[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) { sc[r] = a.bsc[c + r]; sf[r] = a.bsf[c + r]; mu[r] = a.bmu[c + r]; is[r] = a.bis[c + r]; }
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f}, s3[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      if (!valid[j]) continue;
      const int px = px0 + wpx + 16 * j + fr;
      float zv[4];
      ld4(z + (long long)px * a.ldbz + c, zv);
      float d[4] = {1.f, 1.f, 1.f, 1.f};
      if (a.bdrop) {
        const float* dp = a.bdrop + (long long)(px / a.bHW) * a.Cout + c;
#pragma unroll
        for (int r = 0; r < 4; ++r) d[r] = dp[r];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float g = acc[i][j][r];
        if (a.bdrop) g *= d[r];
        if (a.bact == 1 && !(fmaf(zv[r], sc[r], sf[r]) > 0.f)) g = 0.f;
        const float xh = (zv[r] - mu[r]) * is[r];
        s1[r] += g;
        s2[r] = fmaf(g, xh, s2[r]);
        s3[r] += xh;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s1[r] = row16_sum(s1[r]);
      s2[r] = row16_sum(s2[r]);
      s3[r] = row16_sum(s3[r]);
      if (fr == 0) {
        sh[(pw * 3 + 0) * BN + cl + r] = s1[r];
        sh[(pw * 3 + 1) * BN + cl + r] = s2[r];
        sh[(pw * 3 + 2) * BN + cl + r] = s3[r];
      }
    }
  }
  lds_barrier();
  float* row = a.bpart + (long long)(px0 / PXT) * 3 * a.Cout;
  for (int t = tid; t < 3 * BN; t += 512) {  // the pipe / pre-split kernels' 512 threads
    const int k = t / BN, c = t - k * BN;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NPW; ++w) v += sh[(w * 3 + k) * BN + c];
    row[k * a.Cout + co0 + c] = v;
  }
}

__device__ __forceinline__ int swz(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

__device__ __forceinline__ u4v bload(__amdgpu_buffer_rsrc_t r, unsigned off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return __builtin_bit_cast(u4v, v);
}

template <typename T>
__device__ __forceinline__ void mfma_frag(f4v& acc, const u4v& a, const u4v& b) {
  if constexpr (Is16<T>::value) {
    acc = mfma16x16x32<T>(__builtin_bit_cast(s8v, a), __builtin_bit_cast(s8v, b), acc);
  } else {
    // 4 consecutive k of one 16-byte fragment; A and B use the same k order.
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[0]), __uint_as_float(b[0]), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[1]), __uint_as_float(b[1]), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[2]), __uint_as_float(b[2]), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[3]), __uint_as_float(b[3]), acc, 0, 0, 0);
  }
}

// ---------------------------------------------------------------------------
// forward (also used for dgrad with the flipped filter)
// ---------------------------------------------------------------------------
template <typename T, int BCO, int BPX>
__global__ __launch_bounds__(NT, 2) void conv_fwd_kernel(FwdArgs a) {
  constexpr int EPC = 16 / (int)sizeof(T);   // elements per 16-B chunk
  constexpr int BK = 128 / (int)sizeof(T);   // elements per K-tile row
  constexpr int TI = BCO / 32, TJ = BPX / 32;
  constexpr int AR = BCO / 32, BR = BPX / 32;  // rows per thread (8 threads per row)
  constexpr int TILE_BYTES = (BCO + BPX) * 128;
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE_BYTES];

  const int HW = a.H * a.W;
  const int M = a.N * HW;
  const int nco = a.Cout / BCO;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int co0 = (bid % nco) * BCO;
  const int px0 = (bid / nco) * BPX;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int chunk = tid & 7, rbase = tid >> 3;

  // Rebased buffer descriptor over the block's pixel window (halo included).
  const int halo = a.pad * (a.W + 1);
  const int plo = max(0, px0 - halo);
  const int phi = min(M, px0 + BPX + halo);
  const unsigned win_bytes = (unsigned)(((long long)(phi - plo - 1) * a.ldx + a.C) * sizeof(T));
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.x + (long long)plo * a.ldx * sizeof(T)), 0, win_bytes, 0x00020000);

  int pp[BR], pq[BR], prow[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int m = px0 + rbase + 32 * i;
    const int rem = m % HW;
    prow[i] = m;
    pp[i] = (m < M) ? rem / a.W : -100000;
    pq[i] = rem % a.W;
  }

  const int CB = a.C / BK;
  const int KT = a.R * a.S * CB;
  const long long ldw = (long long)a.R * a.S * a.C;
  const T* wp = (const T*)a.w + (long long)(co0 + rbase) * ldw + chunk * EPC;

  u4v ra[AR], rb[BR];
#define FWD_GLOAD(t_) \
  do { \
    const int rs = (t_) / CB, cb = (t_) - rs * CB; \
    const int r = rs / a.S, s = rs - r * a.S; \
    const int coff = cb * BK + chunk * EPC; \
_Pragma("unroll") \
    for (int i = 0; i < AR; ++i) ra[i] = *(const u4v*)(wp + (long long)(32 * i) * ldw + rs * a.C + cb * BK); \
    const int dh = r - a.pad, dw = s - a.pad; \
_Pragma("unroll") \
    for (int i = 0; i < BR; ++i) { \
      const int h = pp[i] + dh, ww = pq[i] + dw; \
      const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)ww < (unsigned)a.W; \
      const long long pin = (long long)(prow[i] + dh * a.W + dw - plo); \
      const unsigned off = ok ? (unsigned)((pin * a.ldx + coff) * (long long)sizeof(T)) : 0xFFFFFFF0u; \
      rb[i] = bload(xr, off); \
    } \
  } while (0)
#define FWD_SWRITE(buf_) \
  do { \
    char* As = smem + (buf_) * TILE_BYTES; \
    char* Bs = As + BCO * 128; \
_Pragma("unroll") \
    for (int i = 0; i < AR; ++i) *(u4v*)(As + swz(rbase + 32 * i, chunk)) = ra[i]; \
_Pragma("unroll") \
    for (int i = 0; i < BR; ++i) *(u4v*)(Bs + swz(rbase + 32 * i, chunk)) = rb[i]; \
  } while (0)
  f4v acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  const int wco = (wid >> 1) * (BCO / 2), wpx = (wid & 1) * (BPX / 2);
  const int fr = lane & 15, fc = lane >> 4;

  FWD_GLOAD(0);
  FWD_SWRITE(0);
  __syncthreads();
  for (int t = 0; t < KT; ++t) {
    const int cur = t & 1;
    if (t + 1 < KT) FWD_GLOAD(t + 1);
    const char* As = smem + cur * TILE_BYTES;
    const char* Bs = As + BCO * 128;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = 4 * ks + fc;
      u4v af[TI], bfr[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) af[i] = *(const u4v*)(As + swz(wco + 16 * i + fr, ch));
#pragma unroll
      for (int j = 0; j < TJ; ++j) bfr[j] = *(const u4v*)(Bs + swz(wpx + 16 * j + fr, ch));
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) mfma_frag<T>(acc[i][j], af[i], bfr[j]);
    }
    if (t + 1 < KT) FWD_SWRITE(cur ^ 1);
    __syncthreads();
  }
#undef FWD_GLOAD
#undef FWD_SWRITE

  // Epilogue: lane holds pixel column fr, 4 consecutive output channels.  Bias, accumulate and
  // the eval-BN affine (all global loads) in a pass of their own ahead of the stores, so the store
  // loop holds no global loads (EPI_ACC_NOTE)
  T* y = (T*)a.y;
  const bool pre = a.bias || a.accumulate || a.escale;
  if (pre) {
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int px = px0 + wpx + 16 * j + fr;
      if (px >= M) continue;
      const T* yrow = y + (long long)px * a.ldy;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int co = co0 + wco + 16 * i + 4 * fc;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if (a.bias) {
          const float4 b = *(const float4*)(a.bias + co);
          v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
        }
        if (a.accumulate) add_old_y(v, yrow, a, px, co);
        epi_affine(v, a, co);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = v[r];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int px = px0 + wpx + 16 * j + fr;
    if (px >= M) continue;
    T* yrow = y + (long long)px * a.ldy;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int co = co0 + wco + 16 * i + 4 * fc;
      const float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      st4(yrow + co, v);
    }
  }
}


// ---------------------------------------------------------------------------
// general implicit GEMM: any R x S, stride, pad (ResNet-50 trunks: 7x7/2 stem via
// im2col, 3x3/2 and 1x1/2 convs), mode 0 = convolution (rows = output pixels
// [N,P,Q] gathering x [N,H,W] at (p*st - pad + r, q*st - pad + s)), mode 1 =
// transposed convolution for dgrad (rows = dX pixels [N,P,Q] gathering dY
// [N,H,W] at ((p + pad - r)/st, (q + pad - s)/st) when divisible).
// The gathered tensor is addressed through one whole-tensor buffer descriptor.
// ---------------------------------------------------------------------------
struct GenArgs {
  const char* x; long long ldx; int N, H, W, C;   // gathered tensor
  int P, Q;                                        // GEMM row grid
  const char* w; int Cout, R, S, stride, pad, mode;
  const float* bias;
  char* y; long long ldy;
  int accumulate;
  // mode 1 with stride > 1: one launch per output parity class (pa, pb): rows are the dX pixels
  // with p % stride == pa, q % stride == pb, and the K loop runs over just the taps that reach
  // them ((p + pad - r) divisible by the stride) -- 1/stride^2 of the taps on average, where the
  // plain transposed gather multiplies zeros for the rest
  int pa = -1, pb = -1;
};

__device__ __forceinline__ bool gen_src(const GenArgs& a, int n, int p, int q, int r, int s, long long& src) {
  int ih, iw;
  if (a.mode == 0) {
    ih = p * a.stride - a.pad + r;
    iw = q * a.stride - a.pad + s;
  } else {
    const int th = p + a.pad - r, tw = q + a.pad - s;
    if (th < 0 || tw < 0) return false;
    ih = th / a.stride; iw = tw / a.stride;
    if (ih * a.stride != th || iw * a.stride != tw) return false;
  }
  if ((unsigned)ih >= (unsigned)a.H || (unsigned)iw >= (unsigned)a.W) return false;
  src = ((long long)n * a.H + ih) * a.W + iw;
  return true;
}

// SPL = 1 (T = float): the f32 GEMM on the bf16 matrix cores through the exact 3-way split of both
// operands per wave (dg_common.h split3_8; conv_fwd_pers_kernel SPL = 1): one 32-channel K-step is
// one 16x16x32 block, the lane's 8 k values being chunks fc and 4 + fc of the 128-B rows
template <typename T, int BCO, int BPX, int SPL = 0>
__global__ __launch_bounds__(NT, 2) void conv_gen_kernel(GenArgs a) {
  constexpr int EPC = 16 / (int)sizeof(T);
  constexpr int BK = 128 / (int)sizeof(T);
  constexpr int TI = BCO / 32, TJ = BPX / 32;
  constexpr int AR = BCO / 32, BR = BPX / 32;
  constexpr int TILE_BYTES = (BCO + BPX) * 128;
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE_BYTES];

  const bool par = a.pa >= 0;  // parity class launch (mode 1, stride > 1)
  const int Pc = par ? (a.P - a.pa + a.stride - 1) / a.stride : a.P;
  const int Qc = par ? (a.Q - a.pb + a.stride - 1) / a.stride : a.Q;
  const int PQ = Pc * Qc;
  const int M = a.N * PQ;
  const int r0 = par ? (a.pa + a.pad) % a.stride : 0, s0 = par ? (a.pb + a.pad) % a.stride : 0;
  const int rst = par ? a.stride : 1;
  const int nr = par ? (a.R - r0 + rst - 1) / rst : a.R, ns = par ? (a.S - s0 + rst - 1) / rst : a.S;
  const int nco = a.Cout / BCO;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int co0 = (bid % nco) * BCO;
  const int px0 = (bid / nco) * BPX;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int chunk = tid & 7, rbase = tid >> 3;

  const unsigned xbytes = (unsigned)((((long long)a.N * a.H * a.W - 1) * a.ldx + a.C) * sizeof(T));
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.x, 0, xbytes, 0x00020000);

  int rn[BR], rp[BR], rq[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int m = px0 + rbase + 32 * i;
    const int rem = m % PQ;
    rn[i] = (m < M) ? m / PQ : -1;
    rp[i] = rem / Qc;
    rq[i] = rem % Qc;
    if (par) {
      rp[i] = rp[i] * a.stride + a.pa;
      rq[i] = rq[i] * a.stride + a.pb;
    }
  }
  const int CB = a.C / BK;
  const int KT = nr * ns * CB;
  const long long ldw = (long long)a.R * a.S * a.C;
  const T* wp = (const T*)a.w + (long long)(co0 + rbase) * ldw + chunk * EPC;

  u4v ra[AR], rb[BR];
#define GEN_GLOAD(t_) \
  do { \
    const int ti = (t_) / CB, cb = (t_) - ti * CB; \
    const int tr = ti / ns; \
    const int r = r0 + rst * tr, s = s0 + rst * (ti - tr * ns); \
    const int rs = r * a.S + s; \
    const int coff = cb * BK + chunk * EPC; \
    _Pragma("unroll") for (int i = 0; i < AR; ++i) ra[i] = *(const u4v*)(wp + (long long)(32 * i) * ldw + rs * a.C + cb * BK); \
    _Pragma("unroll") for (int i = 0; i < BR; ++i) { \
      long long src = 0; \
      const bool ok = rn[i] >= 0 && gen_src(a, rn[i], rp[i], rq[i], r, s, src); \
      const unsigned off = ok ? (unsigned)((src * a.ldx + coff) * (long long)sizeof(T)) : 0xFFFFFFF0u; \
      rb[i] = bload(xr, off); \
    } \
  } while (0)
#define GEN_SWRITE(buf_) \
  do { \
    char* As = smem + (buf_) * TILE_BYTES; \
    char* Bs = As + BCO * 128; \
    _Pragma("unroll") for (int i = 0; i < AR; ++i) *(u4v*)(As + swz(rbase + 32 * i, chunk)) = ra[i]; \
    _Pragma("unroll") for (int i = 0; i < BR; ++i) *(u4v*)(Bs + swz(rbase + 32 * i, chunk)) = rb[i]; \
  } while (0)

  f4v acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  const int wco = (wid >> 1) * (BCO / 2), wpx = (wid & 1) * (BPX / 2);
  const int fr = lane & 15, fc = lane >> 4;

  if (KT > 0) {  // (a parity class no tap reaches, e.g. the odd rows of a 1x1/2 dgrad: zeros)
    GEN_GLOAD(0);
    GEN_SWRITE(0);
  }
  __syncthreads();
  for (int t = 0; t < KT; ++t) {
    const int cur = t & 1;
    if (t + 1 < KT) GEN_GLOAD(t + 1);
    const char* As = smem + cur * TILE_BYTES;
    const char* Bs = As + BCO * 128;
    if constexpr (SPL) {
      static_assert(!Is16<T>::value, "split path is for f32 operands");
      s8v bh[TJ][3];
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const u4v b0 = *(const u4v*)(Bs + swz(wpx + 16 * j + fr, fc));
        const u4v b1 = *(const u4v*)(Bs + swz(wpx + 16 * j + fr, 4 + fc));
        split3_8(b0, b1, bh[j][0], bh[j][1], bh[j][2]);
      }
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const u4v a0 = *(const u4v*)(As + swz(wco + 16 * i + fr, fc));
        const u4v a1 = *(const u4v*)(As + swz(wco + 16 * i + fr, 4 + fc));
        s8v ah[3];
        split3_8(a0, a1, ah[0], ah[1], ah[2]);
        constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
        for (int q = 0; q < 6; ++q)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[PA[q]], bh[j][PB[q]], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int ch = 4 * ks + fc;
        u4v af[TI], bfr[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) af[i] = *(const u4v*)(As + swz(wco + 16 * i + fr, ch));
#pragma unroll
        for (int j = 0; j < TJ; ++j) bfr[j] = *(const u4v*)(Bs + swz(wpx + 16 * j + fr, ch));
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) mfma_frag<T>(acc[i][j], af[i], bfr[j]);
      }
    }
    if (t + 1 < KT) GEN_SWRITE(cur ^ 1);
    __syncthreads();
  }
#undef GEN_GLOAD
#undef GEN_SWRITE
  T* y = (T*)a.y;
  // bias read once and y += old y in a pass of its own, ahead of the stores (EPI_ACC_NOTE)
  f4v bv[TI];
#pragma unroll
  for (int i = 0; i < TI; ++i)
    bv[i] = a.bias ? *(const f4v*)(a.bias + co0 + wco + 16 * i + 4 * fc) : f4v{0.f, 0.f, 0.f, 0.f};
  auto out_row = [&](int px) -> T* {
    long long orow = px;
    if (par) {  // class pixel -> dX pixel (n, stride*i + pa, stride*j + pb)
      const int n = px / PQ, rem = px - n * PQ, i = rem / Qc, jj = rem - i * Qc;
      orow = ((long long)n * a.P + i * a.stride + a.pa) * a.Q + jj * a.stride + a.pb;
    }
    return y + orow * a.ldy;
  };
  if (a.accumulate) {
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int px = px0 + wpx + 16 * j + fr;
      if (px >= M) continue;
      const T* yrow = out_row(px);
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int co = co0 + wco + 16 * i + 4 * fc;
        float o[4];
        ld4(yrow + co, o);
        if (a.bias) {
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += bv[i][r];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] += o[r];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int px = px0 + wpx + 16 * j + fr;
    if (px >= M) continue;
    T* yrow = out_row(px);
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int co = co0 + wco + 16 * i + 4 * fc;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (a.bias && !a.accumulate) {
        const f4v b = bv[i];
        v[0] += b[0]; v[1] += b[1]; v[2] += b[2]; v[3] += b[3];
      }
      st4(yrow + co, v);
    }
  }
}

static bool gen_parity() {  // DGVCC_GEN_PARITY=0: strided dgrad as one transposed gather (A/B switch)
  const char* e = getenv("DGVCC_GEN_PARITY");
  return !(e && e[0] == '0');
}

static bool f32_split();
// DGVCC_GEN_SPLIT=0: f32 strided / general convs on v_mfma_f32_16x16x4_f32 also under the split
// math (read per launch: A/B)
static bool gen_split() {
  const char* e = getenv("DGVCC_GEN_SPLIT");
  return !(e && e[0] == '0');
}

template <typename T>
int launch_gen(const GenArgs& a0, hipStream_t st) {
  bool spl = false;
  if constexpr (!Is16<T>::value) spl = f32_split() && gen_split();
  const int ncls = (a0.mode == 1 && a0.stride > 1 && gen_parity()) ? a0.stride * a0.stride : 1;
  for (int c = 0; c < ncls; ++c) {
    GenArgs a = a0;
    long long M = (long long)a.N * a.P * a.Q;
    if (ncls > 1) {
      a.pa = c / a.stride;
      a.pb = c % a.stride;
      const long long Pc = (a.P - a.pa + a.stride - 1) / a.stride, Qc = (a.Q - a.pb + a.stride - 1) / a.stride;
      M = (long long)a.N * Pc * Qc;
      if (M == 0) continue;
    }
    const int npx = dg_cdiv(M, 128);
    if (spl) {
      if (a.Cout % 128 == 0)
        hipLaunchKernelGGL((conv_gen_kernel<T, 128, 128, !Is16<T>::value>), dim3(npx * (a.Cout / 128)), dim3(NT), 0, st, a);
      else
        hipLaunchKernelGGL((conv_gen_kernel<T, 64, 128, !Is16<T>::value>), dim3(npx * (a.Cout / 64)), dim3(NT), 0, st, a);
    } else if (a.Cout % 128 == 0)
      hipLaunchKernelGGL((conv_gen_kernel<T, 128, 128>), dim3(npx * (a.Cout / 128)), dim3(NT), 0, st, a);
    else
      hipLaunchKernelGGL((conv_gen_kernel<T, 64, 128>), dim3(npx * (a.Cout / 64)), dim3(NT), 0, st, a);
    DG_CHECK_LAUNCH();
  }
  return DG_OK;
}

// transpose (no flip): wt[c][r][s][co] = w[co][r][s][c]
template <typename T>
__global__ void transpose_weight_kernel(const T* __restrict__ w, int Cout, int C, int R, int S, T* __restrict__ wt) {
  const long long total = (long long)Cout * C * R * S;
  for (long long o = blockIdx.x * (long long)blockDim.x + threadIdx.x; o < total;
       o += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(o % Cout);
    long long t = o / Cout;
    const int rs = (int)(t % (R * S));
    const int c = (int)(t / (R * S));
    wt[o] = w[((long long)co * R * S + rs) * C + c];
  }
}

// ---------------------------------------------------------------------------
// bf16 forward, pipelined: 256-pixel x BN-channel tile, 8 waves (4 px x 2 co),
// operands staged global->LDS by LDS-DMA (buffer_load ... lds, 16 B per lane,
// out-of-window taps zero-filled by the descriptor range check) into a 3-stage
// ring with ONE raw barrier per K-step and a counted vmcnt that keeps the next
// K-step's DMA in flight across it (cdna_hip_programming.md §5 "Pipelining across
// barriers").  The XOR swizzle of the 128-B rows is applied on the SOURCE side
// (LDS-DMA destinations are lane-linear): LDS slot p of row r holds global 16-B
// chunk p ^ (r & 7), exactly the image swz() reads.
// ---------------------------------------------------------------------------
constexpr int PBM = 256;   // pixels per tile

// 16-B LDS-DMA: lane l's 16 bytes at voff land at lds + 16*l (wave-uniform base).
// Kept in a __device__ helper: the builtin is not valid in the host pass, which
// would otherwise silently drop the kernel's launch stub.
__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t r, const char* lds, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (DG_LDS void*)lds, 16, voff, 0, 0, 0);
}
// the same with a wave-uniform byte offset added (the instruction's scalar offset operand)
__device__ __forceinline__ void lds_dma16s(__amdgpu_buffer_rsrc_t r, const char* lds, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (DG_LDS void*)lds, 16, voff, soff, 0, 0);
}
constexpr int PSTAGES = 3;

// EPI selects the epilogue at compile time (each variant's registers stay out of the
// others'; runtime branches on all four spilled the 256-wide kernel): 0 = bias / accumulate /
// statistics, 1 = split-K f32 partials, 2 = BN-backward partials (dgrad), 3 = eval BN+ReLU.
template <int BN, int STG, int VAR = 0, int EPI = 0, typename T = bf16>
__global__ __launch_bounds__(512, 1) void conv_fwd_pipe_kernel(FwdArgs a) {
  constexpr int BK = 64;                    // bf16 channels per K-step (128-B rows)
  constexpr int AI = BN / 64;               // A (weight) DMA instructions per wave per K-step
  constexpr int BI = PBM / 64;              // B (pixel) DMA instructions per wave per K-step
  constexpr int TI = BN / 32, TJ = 4;       // wave tile: 64 px x BN/2 co
  constexpr int STAGE = (BN + PBM) * 128;
  constexpr int PF = STG - 1;               // K-steps issued ahead
  __shared__ __attribute__((aligned(1024))) char smem[STG * STAGE];

  const int HW = a.H * a.W;
  const int M = a.N * HW;
  const int nco = a.Cout / BN;
  const int ntile = (M + PBM - 1) / PBM * nco;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / ntile;  // K-slice of a split-K launch (0 otherwise)
  bid -= split * ntile;
  const int co0 = (bid % nco) * BN;
  const int px0 = (bid / nco) * PBM;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lrow = lane >> 3;                          // row within an 8-row DMA group
  const int gchunk = (lane & 7) ^ lrow;                // source chunk landing in slot lane&7

  const int halo = a.pad * (a.W + 1);
  const int plo = max(0, px0 - halo);
  const int phi = min(M, px0 + PBM + halo);
  const unsigned win_bytes = (unsigned)(((long long)(phi - plo - 1) * a.ldx + a.C) * 2);
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.x + (long long)plo * a.ldx * 2), 0, win_bytes, 0x00020000);
  const long long ldw = (long long)a.R * a.S * a.C;
  __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.w + (long long)co0 * ldw * 2), 0, (unsigned)(BN * ldw * 2), 0x00020000);

  // this lane's B rows: pixel (wid*BI + i)*8 + lrow of the tile
  int pp[BI], pq[BI], prow[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int m = px0 + (wid * BI + i) * 8 + lrow;
    const int rem = m % HW;
    prow[i] = m - plo;
    pp[i] = (m < M) ? rem / a.W : -100000;
    pq[i] = rem % a.W;
  }
  unsigned aoff[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) aoff[i] = (unsigned)((((wid * AI + i) * 8 + lrow) * ldw + gchunk * 8) * 2);

  const int CB = a.C / BK;
  const int KTA = a.R * a.S * CB;
  const int kt0 = (int)((long long)split * KTA / a.ksplit);
  const int KT = (int)((long long)(split + 1) * KTA / a.ksplit) - kt0;  // this block's K-steps
  const unsigned cbytes = (unsigned)(gchunk * 16);

#define PIPE_ISSUE(u_, stage_) \
  do { \
    const int kk_ = kt0 + (u_); \
    const int rs = a.korder ? kk_ % (a.R * a.S) : kk_ / CB, cb = a.korder ? kk_ / (a.R * a.S) : kk_ - rs * CB; \
    const int r = rs / a.S, s = rs - r * a.S; \
    char* As = smem + (stage_) * STAGE; \
    char* Bs = As + BN * 128; \
    const unsigned kofs = (unsigned)((rs * a.C + cb * BK) * 2); \
    _Pragma("unroll") for (int i = 0; i < AI; ++i) \
      lds_dma16(wr, As + (wid * AI + i) * 1024, aoff[i] + kofs); \
    const int dh = r - a.pad, dw = s - a.pad; \
    _Pragma("unroll") for (int i = 0; i < BI; ++i) { \
      const int h = pp[i] + dh, ww = pq[i] + dw; \
      const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)ww < (unsigned)a.W; \
      const unsigned off = ok ? (unsigned)(((long long)(prow[i] + dh * a.W + dw) * a.ldx + cb * BK) * 2) + cbytes \
                              : 0xFFFFFFF0u; \
      lds_dma16(xr, Bs + (wid * BI + i) * 1024, off); \
    } \
  } while (0)

  f4v acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  const int wpx = (wid & 3) * 64, wco = (wid >> 2) * (BN / 2);
  const int fr = lane & 15, fc = lane >> 4;

  PIPE_ISSUE(0, 0);
  if (PF > 1 && KT > 1) PIPE_ISSUE(1, 1);
  for (int t = 0; t < KT; ++t) {
    if (PF > 1 && t + 1 < KT) {  // leave step t+1's DMA in flight across the barrier
      if constexpr (AI + BI == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if constexpr (AI + BI == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (VAR != 2 && t + PF < KT) PIPE_ISSUE(t + PF, (t + PF) % STG);
    const char* As = smem + (t % STG) * STAGE;
    const char* Bs = As + BN * 128;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = 4 * ks + fc;
      u4v af[TI], bfr[TJ];
#pragma unroll
      for (int j = 0; j < TJ; ++j) bfr[j] = *(const u4v*)(Bs + swz(wpx + 16 * j + fr, ch));
#pragma unroll
      for (int i = 0; i < TI; ++i) af[i] = *(const u4v*)(As + swz(wco + 16 * i + fr, ch));
      if constexpr (VAR >= 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) mfma_frag<T>(acc[i][j], af[i], bfr[j]);
      if constexpr (VAR >= 1) __builtin_amdgcn_s_setprio(0);
      if constexpr (VAR == 2) {
        if (ks == 0 && t + PF < KT) PIPE_ISSUE(t + PF, (t + PF) % STG);
      }
    }
  }
#undef PIPE_ISSUE

  if constexpr (EPI == 1) {  // raw f32 partial sums of this K-slice
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int px = px0 + wpx + 16 * j + fr;
      if (px >= M) continue;
      float* kp = a.kpart + ((long long)split * M + px) * a.Cout + co0 + wco + 4 * fc;
#pragma unroll
      for (int i = 0; i < TI; ++i) *(f4v*)(kp + 16 * i) = acc[i][j];
    }
    return;
  }
  T* y = (T*)a.y;
  bool valid[TJ];
  // bias read once, ahead of the stores: a load between stores makes the compiler drain vmcnt
  // to 0 per use (the stores may alias it), serialising the tile's stores
  f4v bv[TI];
#pragma unroll
  for (int i = 0; i < TI; ++i)
    bv[i] = a.bias ? *(const f4v*)(a.bias + co0 + wco + 16 * i + 4 * fc) : f4v{0.f, 0.f, 0.f, 0.f};
  if (a.accumulate || EPI == 3) {  // old y, bias and the eval-BN affine ahead of the stores (EPI_ACC_NOTE)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int px = px0 + wpx + 16 * j + fr;
      if (px >= M) continue;
      const T* yrow = y + (long long)px * a.ldy;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int co = co0 + wco + 16 * i + 4 * fc;
        if (a.bias) {
          const f4v b = bv[i];
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += b[r];
        }
        if (a.accumulate) add_old_y(acc[i][j], yrow, a, px, co);
        if constexpr (EPI == 3) {
          float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
          epi_affine(v, a, co);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = v[r];
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int px = px0 + wpx + 16 * j + fr;
    valid[j] = px < M;
    if (px >= M) continue;
    T* yrow = y + (long long)px * a.ldy;
    unsigned pk[2];
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int co = co0 + wco + 16 * i + 4 * fc;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (a.bias && !a.accumulate && EPI != 3) {
        const f4v b = bv[i];
        v[0] += b[0]; v[1] += b[1]; v[2] += b[2]; v[3] += b[3];
      }
      bool stored = false;
      if constexpr (TI % 2 == 0 && EPI == 0) {
        if (a.wide_st & 2) {  // 16-byte stores as in conv_fwd_pers_kernel's WST epilogue
          stored = true;
          if (i % 2 == 0) {
            pk[0] = pack2<T>(v[0], v[1]);
            pk[1] = pack2<T>(v[2], v[3]);
          } else {
            const auto r0 = __builtin_amdgcn_permlane16_swap(pk[0], pack2<T>(v[0], v[1]), false, false);
            const auto r1 = __builtin_amdgcn_permlane16_swap(pk[1], pack2<T>(v[2], v[3]), false, false);
            *(u4v*)(yrow + co0 + wco + 16 * (i - 1) + 8 * (fc >> 1) + 16 * (fc & 1)) = u4v{r0[0], r1[0], r0[1], r1[1]};
          }
        }
      }
      if (!stored) st4(yrow + co, v);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = round_to<T>(v[r]);  // the stored value, for the statistics
    }
  }
  if constexpr (EPI == 0) {
    if (a.part)
      epi_stats<TI, TJ, 4, BN>(acc, valid, wid & 3, wco, smem, a.part + (long long)(px0 / PBM) * 3 * a.Cout, a.Cout,
                               co0, tid, fr, fc);
  }
  if constexpr (EPI == 2) epi_bnbwd<TI, TJ, 4, BN, T>(acc, valid, wid & 3, wco, wpx, smem, a, px0, co0, tid, fr, fc);
}

// Persistent form of conv_fwd_pipe_kernel (VAR 2 schedule): one block per CU walks its
// tiles (block b, tiles b, b + G, ... through the same XCD remap) and keeps the LDS-DMA
// ring running across tile boundaries: the next tile's first K-steps are issued during
// the current tile's last ones, so its prologue latency hides under the current tile's
// MFMAs and epilogue stores.  The epilogue-statistics scratch gets its own LDS so the
// in-flight ring stages are never touched.  Requires KT > PF (K-steps per tile).
constexpr int PERS_BIAS_MAX = 1024;  // Cout limit of the persistent forward (LDS bias)
// SPL = 1 (T = float only): the f32 GEMM on the bf16 matrix cores through the exact 3-way
// split (dg_common.h split3_8): one 32-channel K-step is one 16x16x32 block, the lane's 8
// k values being its chunks fc and 4 + fc of the 128-B row for both operands.
// Tap validity of the B (pixel) DMA pieces of a persistent conv tile, for the incremental
// addressing (INC): the image-bounds test of tap (r, s) is separable, so each piece keeps 6 bits,
// rows r = 0..2 at bits 0..2 and columns s = 0..2 at bits 3..5, five pieces per 32-bit word
// (R, S <= 3).  Tap (r, s) of piece i is inside the image iff both of need(r, s) << 6 (i % 5) are set.
template <int BI>
struct TapMask {
  unsigned w[(BI + 4) / 5];
};
template <int BI>
__device__ __forceinline__ void tapmask_set(TapMask<BI>& t, int i, int pp, int pq, const FwdArgs& a) {
  if (i % 5 == 0) t.w[i / 5] = 0;
  unsigned b = 0;
  for (int r = 0; r < a.R; ++r) b |= ((unsigned)(pp + r - a.pad) < (unsigned)a.H) ? 1u << r : 0u;
  for (int s2 = 0; s2 < a.S; ++s2) b |= ((unsigned)(pq + s2 - a.pad) < (unsigned)a.W) ? 8u << s2 : 0u;
  t.w[i / 5] |= b << (6 * (i % 5));
}
__device__ __forceinline__ unsigned tap_need(int r, int s2) { return (1u << r) | (8u << s2); }
template <int BI>
__device__ __forceinline__ bool tapmask_ok(const TapMask<BI>& t, int i, unsigned need) {
  const unsigned nd = need << (6 * (i % 5));
  return (t.w[i / 5] & nd) == nd;
}

// INC: incremental DMA addressing as in conv_fwd_psplit_kernel (DGVCC_PERS_INC=0 restores the per-K-step
// recomputation)
// WIDE (16-bit, BN = 128): 384-pixel tiles with the 8 waves all on pixels, each 128 channels x 48
// pixels (the 256-channel kernel's per-wave filter reuse; 1.5x the MFMAs per barrier of the 2 x 4
// layout of 64 x 64 wave tiles), two stages of (16 + 48) KB (DGVCC_PERS_WIDE=0: the 2 x 4 layout).
template <int BN, int STG, int EPI = 0, typename T = bf16, int SPL = 0, int INC = 1, int WIDE = 0, int WST = 0>
__global__ __launch_bounds__(512, 1) void conv_fwd_pers_kernel(FwdArgs a) {
  static_assert(!WIDE || (BN == 128 && SPL == 0 && STG == 2), "WIDE: the 16-bit 128-channel kernel");
  constexpr int PB = WIDE ? 384 : PBM;   // pixels per tile
  constexpr int NPXG = WIDE ? 8 : 4;     // pixel groups of waves
  constexpr int NCOG = 8 / NPXG;         // channel groups of waves
  constexpr int ES = (int)sizeof(T);  // element bytes: a K-step row is 128 B (64 x 16-bit or 32 x f32)
  constexpr int BK = 128 / ES;
  constexpr int AI = BN / 64;
  constexpr int BI = PB / 64;
  constexpr int TI = BN / NCOG / 16, TJ = PB / NPXG / 16;
  constexpr int STAGE = (BN + PB) * 128;
  constexpr int PF = STG - 1;
  constexpr int EPI_B = NPXG * 3 * BN * 4;  // epi_stats scratch [NPXG][3][BN] f32
  __shared__ __attribute__((aligned(1024))) char smem[STG * STAGE + EPI_B + PERS_BIAS_MAX * 4];
  char* epi_lds = smem + STG * STAGE;
  // bias staged in LDS once per block: a global load per use in the epilogue makes the
  // compiler drain vmcnt to 0, i.e. wait for the next tile's in-flight DMA steps and every
  // earlier store of the tile (vector-memory operations retire in issue order)
  float* bbuf = (float*)(epi_lds + EPI_B);
  // eval BN (EPI 3, no statistics scratch needed): bias, scale and shift all staged in LDS
  // (the statistics scratch + bias region, 3 x Cout floats) when they fit, else global loads
  constexpr int E3_MAX = (EPI_B + PERS_BIAS_MAX * 4) / 12;
  const bool e3_lds = EPI == 3 && a.Cout <= E3_MAX;
  float* ebias = (float*)epi_lds;
  float* escl = ebias + E3_MAX;
  float* eshf = escl + E3_MAX;

  const int HW = a.H * a.W;
  const int M = a.N * HW;
  const int nco = a.Cout / BN;
  const int ntile = (M + PB - 1) / PB * nco;
  const int G = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lrow = lane >> 3;
  const int gchunk = (lane & 7) ^ lrow;
  const long long ldw = (long long)a.R * a.S * a.C;
  const int CB = a.C / BK;
  const int KT = a.R * a.S * CB;
  const unsigned cbytes = (unsigned)(gchunk * 16);
  unsigned aoff[AI];
#pragma unroll
  for (int i = 0; i < AI; ++i) aoff[i] = (unsigned)(((wid * AI + i) * 8 + lrow) * ldw * ES + gchunk * 16);

  struct Ctx {
    int px0, co0;
    __amdgpu_buffer_rsrc_t xr, wr;
    int pp[BI], pq[BI], prow[BI];
    unsigned bofs;        // INC: piece 0's window byte offset (piece i: + 8 i rows)
    TapMask<BI> tm;       // INC: the pieces' in-image taps
  };
  auto setup = [&](int lin, Ctx& c) {
    const int t = xcd_remap(lin, ntile);
    c.co0 = (t % nco) * BN;
    c.px0 = (t / nco) * PB;
    const int halo = a.pad * (a.W + 1);
    const int plo = max(0, c.px0 - halo);
    const int phi = min(M, c.px0 + PB + halo);
    const unsigned win_bytes = (unsigned)(((long long)(phi - plo - 1) * a.ldx + a.C) * ES);
    c.xr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.x + (long long)plo * a.ldx * ES), 0, win_bytes, 0x00020000);
    c.wr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.w + (long long)c.co0 * ldw * ES), 0, (unsigned)(BN * ldw * ES),
                                             0x00020000);
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int m = c.px0 + (wid * BI + i) * 8 + lrow;
      const int rem = m % HW;
      c.prow[i] = m - plo;
      c.pp[i] = (m < M) ? rem / a.W : -100000;
      c.pq[i] = rem % a.W;
      if constexpr (INC) {
        if (i == 0) c.bofs = (unsigned)((long long)c.prow[0] * a.ldx * ES) + cbytes;
        tapmask_set<BI>(c.tm, i, c.pp[i], c.pq[i], a);
      }
    }
  };
  const int RS = a.R * a.S;
  // INC: the K-step of the next DMA issue as three digits, fastest first: (s, r, cb) in the
  // channel-block-major order (a.korder), (cb, s, r) in the tap-major one
  const bool ko = a.korder != 0;
  const int L0 = ko ? a.S : CB, L1 = ko ? a.R : a.S;
  int d0 = 0, d1 = 0, d2 = 0;
  auto issue_inc = [&](const Ctx& c, unsigned stage) {
    const int is = ko ? d0 : d1, ir = ko ? d1 : d2, icb = ko ? d2 : d0;
    const int rs = ir * a.S + is;
    char* As = smem + stage * STAGE;
    char* Bs = As + BN * 128;
    const unsigned kofs = (unsigned)((rs * a.C + icb * BK) * ES);
#pragma unroll
    for (int i = 0; i < AI; ++i) lds_dma16(c.wr, As + (wid * AI + i) * 1024, aoff[i] + kofs);
    const unsigned toff = (unsigned)((((ir - a.pad) * a.W + (is - a.pad)) * a.ldx + icb * BK) * ES);
    const unsigned need = tap_need(ir, is);
#pragma unroll
    for (int i = 0; i < BI; ++i)
      lds_dma16(c.xr, Bs + (wid * BI + i) * 1024,
                tapmask_ok<BI>(c.tm, i, need) ? c.bofs + (toff + (unsigned)(i * 8 * a.ldx * ES)) : 0xFFFFFFF0u);
    d0 += 1;
    if (d0 == L0) {
      d0 = 0;
      d1 += 1;
      if (d1 == L1) {
        d1 = 0;
        d2 += 1;
      }
    }
  };
  // the step PF ahead of consumed step t, possibly the next tile's
  auto issue_ahead = [&](const Ctx& c, const Ctx& n, int t, bool hn, unsigned stage) {
    const int u = t + PF;
    if constexpr (INC) {
      if (u < KT) issue_inc(c, stage);
      else if (hn) {
        if (u == KT) d0 = d1 = d2 = 0;
        issue_inc(n, stage);
      }
    }
  };
  auto issue = [&](const Ctx& c, int kt, int stage) {
    const int rs = a.korder ? kt % RS : kt / CB, cb = a.korder ? kt / RS : kt - rs * CB;
    const int r = rs / a.S, s2 = rs - r * a.S;
    char* As = smem + stage * STAGE;
    char* Bs = As + BN * 128;
    const unsigned kofs = (unsigned)((rs * a.C + cb * BK) * ES);
#pragma unroll
    for (int i = 0; i < AI; ++i) lds_dma16(c.wr, As + (wid * AI + i) * 1024, aoff[i] + kofs);
    const int dh = r - a.pad, dw = s2 - a.pad;
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int hh = c.pp[i] + dh, ww = c.pq[i] + dw;
      const bool ok = (unsigned)hh < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
      const unsigned off =
          ok ? (unsigned)(((long long)(c.prow[i] + dh * a.W + dw) * a.ldx + cb * BK) * ES) + cbytes : 0xFFFFFFF0u;
      lds_dma16(c.xr, Bs + (wid * BI + i) * 1024, off);
    }
  };

  int lin = blockIdx.x;
  if (lin >= ntile) return;
  if (e3_lds) {
    for (int c = tid; c < a.Cout; c += 512) {
      ebias[c] = a.bias ? a.bias[c] : 0.f;
      escl[c] = a.escale[c];
      eshf[c] = a.eshift[c];
    }
  } else if (a.bias) {
    for (int c = tid; c < a.Cout; c += 512) bbuf[c] = a.bias[c];
  }
  Ctx cur, nxt;
  setup(lin, cur);
  bool has_next = lin + G < ntile;
  if (has_next) setup(lin + G, nxt);
  const int wpx = (wid % NPXG) * (PB / NPXG), wco = (wid / NPXG) * (BN / NCOG);
  const int fr = lane & 15, fc = lane >> 4;
  unsigned gs = 0;  // K-steps issued/consumed across all tiles of this block
  if constexpr (INC) {
    issue_inc(cur, 0);
    if (PF > 1) issue_inc(cur, 1);
  } else {
    issue(cur, 0, 0);
    if (PF > 1) issue(cur, 1, 1);
  }
  bool first_tile = true;
  while (true) {
    f4v acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < KT; ++t, ++gs) {
      const bool more = t + 1 < KT || has_next;
      if (PF > 1 && more && (t > 0 || first_tile)) {  // leave the next step's DMA in flight
        if constexpr (AI + BI == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else if constexpr (AI + BI == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {  // (after an epilogue its stores are the youngest operations: drain everything)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const char* As = smem + (gs % STG) * STAGE;
      const char* Bs = As + BN * 128;
      if constexpr (SPL) {
        static_assert(!Is16<T>::value, "split path is for f32 operands");
        u4v b0[TJ], b1[TJ];
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          b0[j] = *(const u4v*)(Bs + swz(wpx + 16 * j + fr, fc));
          b1[j] = *(const u4v*)(Bs + swz(wpx + 16 * j + fr, 4 + fc));
        }
        // A fragments one row block ahead of their MFMAs (all TI at once spill at BN = 256)
        u4v a0 = *(const u4v*)(As + swz(wco + fr, fc)), a1 = *(const u4v*)(As + swz(wco + fr, 4 + fc));
        if constexpr (INC) issue_ahead(cur, nxt, t, has_next, (gs + PF) % STG);
        else {  // the step PF ahead (its stage was last read before this step's barrier)
          const int u = t + PF;
          if (u < KT) issue(cur, u, (gs + PF) % STG);
          else if (has_next) issue(nxt, u - KT, (gs + PF) % STG);
        }
        s8v bh[TJ][3];
#pragma unroll
        for (int j = 0; j < TJ; ++j) split3_8(b0[j], b1[j], bh[j][0], bh[j][1], bh[j][2]);
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          s8v ah[3];
          split3_8(a0, a1, ah[0], ah[1], ah[2]);
          if (i + 1 < TI) {
            a0 = *(const u4v*)(As + swz(wco + 16 * (i + 1) + fr, fc));
            a1 = *(const u4v*)(As + swz(wco + 16 * (i + 1) + fr, 4 + fc));
          }
          __builtin_amdgcn_s_setprio(1);
          constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
          for (int q = 0; q < 6; ++q)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[PA[q]], bh[j][PB[q]], acc[i][j], 0, 0, 0);
          __builtin_amdgcn_s_setprio(0);
        }
        continue;
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int ch = 4 * ks + fc;
        u4v af[TI], bfr[TJ];
#pragma unroll
        for (int j = 0; j < TJ; ++j) bfr[j] = *(const u4v*)(Bs + swz(wpx + 16 * j + fr, ch));
#pragma unroll
        for (int i = 0; i < TI; ++i) af[i] = *(const u4v*)(As + swz(wco + 16 * i + fr, ch));
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) mfma_frag<T>(acc[i][j], af[i], bfr[j]);
        __builtin_amdgcn_s_setprio(0);
        if (ks == 0) {  // the step PF ahead, possibly the next tile's
          if constexpr (INC) issue_ahead(cur, nxt, t, has_next, (gs + PF) % STG);
          else {
            const int u = t + PF;
            if (u < KT) issue(cur, u, (gs + PF) % STG);
            else if (has_next) issue(nxt, u - KT, (gs + PF) % STG);
          }
        }
      }
    }
    first_tile = false;
    // epilogue of the current tile (the next tile's first DMAs are in flight)
    T* y = (T*)a.y;
    bool valid[TJ];
    // y += old y ahead of the stores (EPI_ACC_NOTE)
    if (a.accumulate) {
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int px = cur.px0 + wpx + 16 * j + fr;
        if (px >= M) continue;
        const T* yrow = y + (long long)px * a.ldy;
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int co = cur.co0 + wco + 16 * i + 4 * fc;
          if (e3_lds) {
            const f4v b = *(const f4v*)(ebias + co);
            for (int r = 0; r < 4; ++r) acc[i][j][r] += b[r];
          } else if (a.bias) {
            const f4v b = *(const f4v*)(bbuf + co);
            for (int r = 0; r < 4; ++r) acc[i][j][r] += b[r];
          }
          add_old_y(acc[i][j], yrow, a, px, co);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int px = cur.px0 + wpx + 16 * j + fr;
      valid[j] = px < M;
      if (px >= M) continue;
      T* yrow = y + (long long)px * a.ldy;
      unsigned pk[2];  // wide stores: this lane's packed group i (even) until group i + 1 is ready
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int co = cur.co0 + wco + 16 * i + 4 * fc;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if (a.accumulate) {
        } else if (e3_lds) {
          const f4v b = *(const f4v*)(ebias + co);
          v[0] += b[0]; v[1] += b[1]; v[2] += b[2]; v[3] += b[3];
        } else if (a.bias) {
          const f4v b = *(const f4v*)(bbuf + co);
          v[0] += b[0]; v[1] += b[1]; v[2] += b[2]; v[3] += b[3];
        }
        if constexpr (EPI == 3) {
          if (e3_lds) {  // same fmaf / ReLU as epi_affine on the same f32 value
            const f4v sc = *(const f4v*)(escl + co), sf = *(const f4v*)(eshf + co);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float tt = fmaf(v[r], sc[r], sf[r]);
              if (a.eact == 1) tt = tt > 0.f ? tt : 0.f;
              v[r] = tt;
            }
          } else {
            epi_affine(v, a, co);
          }
        }
        bool stored = false;
        if constexpr (WST && Is16<T>::value && TI % 2 == 0) {
          // Lane (fr, fc) holds channels 16i + 4fc .. +3 of pixel fr.  v_permlane16_swap of the
          // packed groups i (vdst) and i + 1 (src) swaps rows 1 / 3 of vdst with rows 0 / 2 of src,
          // so fc = 0 / 2 end with channels 16i + 8(fc/2) .. +7 and fc = 1 / 3 with the same of
          // group i + 1: one 16-byte store per lane per group pair (the lane pairs share fr, so
          // share px and the bounds check), 16 rows x 64 contiguous bytes per instruction
          {
            stored = true;
            if (i % 2 == 0) {
              pk[0] = pack2<T>(v[0], v[1]);
              pk[1] = pack2<T>(v[2], v[3]);
            } else {
              const auto r0 = __builtin_amdgcn_permlane16_swap(pk[0], pack2<T>(v[0], v[1]), false, false);
              const auto r1 = __builtin_amdgcn_permlane16_swap(pk[1], pack2<T>(v[2], v[3]), false, false);
              *(u4v*)(yrow + cur.co0 + wco + 16 * (i - 1) + 8 * (fc >> 1) + 16 * (fc & 1)) =
                  u4v{r0[0], r1[0], r0[1], r1[1]};
            }
          }
        }
        if (!stored) st4(yrow + co, v);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = round_to<T>(v[r]);
      }
    }
    if (EPI == 0 && a.part)
      epi_stats<TI, TJ, NPXG, BN>(acc, valid, wid % NPXG, wco, epi_lds, a.part + (long long)(cur.px0 / PB) * 3 * a.Cout,
                               a.Cout, cur.co0, tid, fr, fc);
    if (!has_next) break;
    cur = nxt;
    lin += G;
    has_next = lin + G < ntile;
    if (has_next) setup(lin + G, nxt);
  }
}

// f32 forward/dgrad on the bf16 matrix cores with the filter panel PRE-SPLIT (dg_common.h
// split3_8 applied once per launch by split_weight_kernel, not per wave per K-step): the A
// operand arrives by LDS-DMA as three bf16 planes [part][BN rows][32 channels] (64-B rows,
// 16-B chunk c of row r stored at c ^ psw_a(r): conflict-free fragment reads), the
// f32 pixel rows as in conv_fwd_pers_kernel; only the B (pixel) fragments are split in
// registers.  192-pixel tiles (8 waves = 4 pixel x 2 channel, 48 x BN/2 each): the planes
// make a K-step's A tile 1.5x the f32 bytes, and 2 x (48 + 24) KB + epilogue scratch fill
// the 160-KB LDS exactly at BN = 256.  k order within a 32-channel block: lane group fc
// holds channels 8fc..8fc+7 for both operands.
// LDS swizzles of the pre-split kernel, conflict-free for gfx950's ds_read_b128 lane groups
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ... : MI355X_MICROARCH.md LDS table), with lane
// (fr = lane & 15, fc = lane >> 4) reading row base + fr (base a multiple of 16):
//  * 64-B bf16 plane rows (4 per 256-B bank window; the filter planes here and in the Cout = 64
//    kernels, whose 3-tap strips are also read at row offsets 1 and 2): logical chunk c of row r
//    at c ^ psw_a(r & 15), psw_a = 2 on rows {4, 5, 10..15} and 0 elsewhere, conflict-free at row
//    offsets 0, 1 and 2 (found by exhaustive search; the linear (r >> 2) & 3 put rows r and r + 4
//    of one lane group on the same banks: 2-way on every fragment read);
//  * B pixel rows (f32, 128 B, 2 per window), chunks 2fc and 2fc + 1: c ^ psw_b(r & 15), psw_b
//    splitting rows {0-3, 12-15} and {4-11} (the two halves of a lane group) into chunk
//    quartets 0-3 / 4-7 (r & 7 was 2-way as well).
// Checked exhaustively over the lane groups; SQ_LDS_BANK_CONFLICT on the 512 -> 512 layer was
// 5.7e8 cycles per launch before.
__device__ __forceinline__ int psw_a(int r) { return (0xaaa00a00u >> ((r & 15) * 2)) & 3; }
__device__ __forceinline__ int psw_b(int r) {
  return ((((r >> 3) ^ (r >> 2)) & 1) << 2) | (((r >> 3) & 1) << 1) | ((r >> 1) & 1);
}
__device__ __forceinline__ int swzb(int row, int chunk) { return row * 128 + ((chunk ^ psw_b(row & 15)) << 4); }

constexpr int PSB = 192;  // pixels per tile of the pre-split kernel at BN = 256
// BN = 128: 384-pixel tiles with the 8 waves all on pixels (each 128 channels x 48 pixels, the
// BN = 256 kernel's wave tile), two stages of (24 + 48) KB: the filter fragments are reused by 8
// waves instead of 4 (the 192-pixel 2 x 4 layout ran 52% MFMA-busy against 65% at BN = 256)
__host__ __device__ constexpr int psplit_psb(int BN, int wide = 1) { return BN == 128 && wide ? 384 : PSB; }
static bool psplit_wide() {  // DGVCC_PSPLIT_WIDE=0: BN = 128 on 192-pixel tiles of 2 x 4 waves
  const char* e = getenv("DGVCC_PSPLIT_WIDE");
  return !(e && e[0] == '0');
}
static bool pers_inc() {  // DGVCC_PERS_INC=0: the persistent 16-bit forward with per-K-step addressing (A/B)
  const char* e = getenv("DGVCC_PERS_INC");
  return !(e && e[0] == '0');
}
// the incremental addressing's tap masks hold R, S <= 3
static bool inc_shape_ok(const FwdArgs& a) { return a.R <= 3 && a.S <= 3; }
static bool psplit_inc() {  // DGVCC_PSPLIT_INC=0: per-K-step recomputed DMA addressing (read per launch: A/B)
  const char* e = getenv("DGVCC_PSPLIT_INC");
  return !(e && e[0] == '0');
}
// INC = 1: the DMA of each K-step is addressed incrementally.  The issue cursor (r, s, cb) steps
// through the K order without divisions, and each B piece keeps its tile-constant window byte
// offset plus a bit mask of the taps that stay inside the image (bit r * S + s), so a K-step's
// B offsets are one scalar tap/channel offset added per piece.  INC = 0 (DGVCC_PSPLIT_INC=0)
// recomputes kt -> (rs, cb) and each piece's bounds check and offset at every K-step: ~130
// scalar and ~30 vector instructions in front of the split on every wave.
// TALL = 1 (BN = 256, EPI 0): 256-pixel tiles, each wave 128 channels x 64 pixels (TJ = 4), so every
// filter fragment read and every staged filter byte feeds 4 pixel blocks instead of 3.  The two
// 80-KB stages fill the LDS; the epilogue's statistics scratch and this tile's bias live in the
// stage the last K-step consumed (free until the next tile's second K-step issues its DMA there).
// HM = 1: the f16 x3 arithmetic (dg_common.h split2h_8 / mfma_h3): two f16 filter planes
// (split_weight_h_kernel: per-row scale, 1/(s_row s_x) per output channel after the planes, then
// s_x), the pixel fragments scaled by s_x and split into two f16 parts, three MFMAs per block.
// STAMP = 1: diagnostic build (DGVCC_PSPLIT_STAMP with dg_debug_stamps' buffer): s_memtime stamps around
// each K-step's phases -- DMA wait, barrier, prologue (fragment reads, next DMA issue, B split), MFMA
// block -- and the epilogue, summed per wave and stored once at the end (cdna_hip_programming.md §7
// "In-kernel stamps"; read its shares, not its run time).
// SCH (HM only): 0 = the next K-step's DMA issued in the prologue (after the first fragment reads), every
// MFMA block at s_setprio 1; 1 = its AI + BI pieces issued one per MFMA block (i < AI + BI), so the
// prologue ahead of the first MFMA is reads + split only; 2 = 1 with a static s_setprio 1 for waves
// 4-7 (the arbitration losers of the 8-wave block) and no per-block priority flips; 3 = SIMD partners
// out of phase: waves 0-3 issue their DMA in the prologue (as 0) while waves 4-7 run their MFMA block,
// and waves 4-7 issue theirs after their MFMA block while waves 0-3 run theirs (an LDS-DMA piece costs its
// wave 100-185 issue cycles, MI355X_MICROARCH.md); 4 = 3 without the per-block s_setprio; 5 (TALL, KT >= 2):
// register staging instead of LDS-DMA -- each K-step's A and B pieces are loaded into registers
// (buffer_load_dwordx4, the same addresses and out-of-window zero fill) two K-steps ahead and stored
// to their stage with ds_write_b128 one K-step ahead, after the current stage's fragment reads; the
// stage is then ordered by lgkmcnt + the barrier instead of vmcnt.  The same LDS image and MFMA
// order: bit-identical to SCH 0.  6 (TALL, HM): the two channel halves' waves (0-3: channels 0-127, 4-7:
// 128-255; SIMD partners) one phase apart, two barriers per K-step: in phase 1 of K-step t waves 0-3
// read and split K-step t's fragments while waves 4-7 run their MFMA block of K-step t - 1; in phase 2
// every wave issues K-step t + 1's DMA (into the stage K-step t - 1 freed), waves 0-3 run their MFMA
// block of K-step t and waves 4-7 read and split K-step t's fragments.  Each SIMD then holds one wave
// in its MFMA block and one in its prologue, where SCH 0 keeps both in the same phase (the stamp build
// put their prologues at 28% / 66% of the K-step).  A tile ends with a drain phase (waves 4-7's last
// MFMA block) before the shared epilogue.  The same fragments and MFMA order: bit-identical to SCH 0.
template <int BN, int STG, int EPI = 0, int WIDE = 1, int INC = 1, int TALL = 0, int HM = 0, int STAMP = 0,
          int SCH = 0>
__global__ __launch_bounds__(512, 1) void conv_fwd_psplit_kernel(FwdArgs a, const char* __restrict__ wsp) {
  static_assert(!TALL || (BN == 256 && EPI == 0 && STG == 2 && INC), "TALL: 256-channel training forward only");
  static_assert(SCH != 5 || (TALL && HM), "SCH 5: the TALL f16 x3 kernel");
  static_assert(SCH != 6 || (TALL && HM && STG == 2 && !STAMP), "SCH 6: the TALL f16 x3 kernel");
  static_assert(SCH != 7 || (TALL && HM), "SCH 7: diagnostic timing of the TALL f16 x3 kernel without the split");
  // SCH 8 (HM): the pixel operand arrives PRE-SPLIT (split_x_h_kernel, once per launch): a.x is the
  // [M][C/32][hi 32 x f16 | lo 32 x f16] image of x * s_x, the same 128 B per (pixel, 32-channel block)
  // as the f32 rows, so the DMA is unchanged and the prologue reads the two parts' chunks fc and 4 + fc
  // instead of splitting (the split was 28% of the kernel: SCH 7).  Bit-identical to SCH 0.
  static_assert(SCH != 8 || HM, "SCH 8: the f16 x3 kernels");
  // SCH 9 (TALL, HM): the split once per block instead of once per wave.  The two waves of a pixel group
  // (its two 128-channel halves) split the same B fragments under SCH 0; here each converts half of the
  // group's stage rows in place into the SCH 8 image (hi chunks 0-3, lo chunks 4-7 of the 128-B row:
  // every lane reads its row's two f32 chunks, the four lanes of a row in one instruction, before any
  // writes) and, after a second barrier, the K-step reads the parts as SCH 8 does.  Half the split VALU
  // per wave for an LDS round trip of the stage's B bytes and one barrier; bit-identical to SCH 0.
  static_assert(SCH != 9 || (TALL && HM && !STAMP), "SCH 9: the TALL f16 x3 kernel");
  constexpr bool PRE = SCH == 8 || SCH == 9;  // the K-step reads the pre-split image
  constexpr bool RSTG = SCH == 5;
  constexpr int NPL = HM ? 2 : 3;  // filter planes
  constexpr int KB = NPL * 64;     // bytes per (output channel, 32-deep k-block) of the planes
  constexpr int PSB = TALL ? 256 : psplit_psb(BN, WIDE);
  constexpr int NCOG = (BN == 128 && WIDE) ? 1 : 2;  // channel groups of waves
  constexpr int NPXG = 8 / NCOG;                   // pixel groups of waves
  constexpr int AROWB = 64;                        // bytes per A plane row (32 bf16)
  constexpr int A_BYTES = NPL * BN * AROWB;
  constexpr int AI = A_BYTES / 1024 / 8;           // A DMA instructions per wave per K-step
  constexpr int BI = PSB / 64;                     // B DMA instructions per wave per K-step
  constexpr int TI = BN / NCOG / 16, TJ = PSB / NPXG / 16;  // wave tile: 128 channels x 48 pixels
  constexpr int STAGE = A_BYTES + PSB * 128;
  constexpr int PF = STG - 1;
  constexpr int EPI_B = NPXG * 3 * BN * 4;
  static_assert(AI * 8 * 1024 == A_BYTES, "A tile must split evenly over the 8 waves");
  // non-TALL: epilogue scratch, the bias row and (HM) the per-channel rescale row after the ring
  __shared__ __attribute__((aligned(1024))) char smem[STG * STAGE + (TALL ? 0 : EPI_B + PERS_BIAS_MAX * 4 * (HM ? 2 : 1))];
  static_assert(!TALL || EPI_B + (HM ? 2 : 1) * BN * 4 <= STAGE, "TALL epilogue scratch must fit in a stage");
  char* epi_lds = smem + STG * STAGE;
  float* bbuf = (float*)(epi_lds + EPI_B);
  float* hbuf = bbuf + PERS_BIAS_MAX;  // HM: the rescale exponents -(e_row + e_x) (int bits) by absolute output channel
  constexpr int E3_MAX = (EPI_B + PERS_BIAS_MAX * 4) / 12;
  const bool e3_lds = EPI == 3 && a.Cout <= E3_MAX;
  float* ebias = (float*)epi_lds;
  float* escl = ebias + E3_MAX;
  float* eshf = escl + E3_MAX;

  const int HW = a.H * a.W;
  const int M = a.N * HW;
  const int nco = a.Cout / BN;
  const int ntile = (M + PSB - 1) / PSB * nco;
  const int G = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lrow = lane >> 3;
  const int CB = a.C / 32;
  const int KT = a.R * a.S * CB;
  unsigned cbytes[BI];  // B DMA source chunk of this lane for piece i (rows (wid * BI + i) * 8 + lrow)
#pragma unroll
  for (int i = 0; i < BI; ++i) cbytes[i] = (unsigned)(((lane & 7) ^ psw_b((((wid * BI + i) & 1) << 3) + lrow)) * 16);
  // A source offsets (bytes, K-step 0) of this wave's AI DMA pieces: piece q = plane p, rows rb*16..+15
  // = a lane part (row (lane >> 2) of a 16-row block; the swizzle only sees row & 15) + a
  // wave-uniform part per piece (scalar offset of the DMA), so the pieces cost one VGPR
  const unsigned alane = (unsigned)((lane >> 2) * KT * KB + (((lane & 3) ^ psw_a(lane >> 2)) * 16));
  // HM: the scales after the planes: [Cout] the rescale exponents -(e_row + e_x) (int bits), then s_x
  const float* htail = (const float*)(wsp + (long long)a.Cout * KT * KB);
  const float hsx = HM ? htail[a.Cout] : 1.f;
  auto aoff_s = [&](int q) -> unsigned {
    const int gq = wid * AI + q;
    const int pl = gq / (BN / 16), rb = gq % (BN / 16);
    return (unsigned)(rb * 16 * KT * KB + pl * 64);
  };

  struct Ctx {
    int px0, co0;
    __amdgpu_buffer_rsrc_t xr, wr;
    int pp[BI], pq[BI], prow0;  // INC = 0: piece i's window row: prow0 + 8 i
    unsigned bofs;        // INC = 1: window byte offset of piece 0's row (piece i: + 8 i rows + its chunk)
    TapMask<BI> tm;       // INC = 1: the pieces' in-image taps
  };
  auto setup = [&](int lin, Ctx& c) {
    const int t = xcd_remap(lin, ntile);
    if (a.tile_order) {  // channel-tile-major: an XCD's concurrent tiles share one filter panel
      const int npx = ntile / nco;
      c.co0 = (t / npx) * BN;
      c.px0 = (t - (t / npx) * npx) * PSB;
    } else {
      c.co0 = (t % nco) * BN;
      c.px0 = (t / nco) * PSB;
    }
    const int halo = a.pad * (a.W + 1);
    const int plo = max(0, c.px0 - halo);
    c.prow0 = c.px0 + wid * BI * 8 + lrow - plo;
    const int phi = min(M, c.px0 + PSB + halo);
    const unsigned win_bytes = (unsigned)(((long long)(phi - plo - 1) * a.ldx + a.C) * 4);
    c.xr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.x + (long long)plo * a.ldx * 4), 0, win_bytes, 0x00020000);
    c.wr = __builtin_amdgcn_make_buffer_rsrc((void*)(wsp + (long long)c.co0 * KT * KB), 0, (unsigned)(BN * KT * KB),
                                             0x00020000);
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int m = c.px0 + (wid * BI + i) * 8 + lrow;
      const int rem = m % HW;
      c.pp[i] = (m < M) ? rem / a.W : -100000;
      c.pq[i] = rem % a.W;
      if constexpr (INC) {
        if (i == 0) c.bofs = (unsigned)((long long)c.prow0 * a.ldx * 4);
        tapmask_set<BI>(c.tm, i, c.pp[i], c.pq[i], a);
      }
    }
  };
  const int RS = a.R * a.S;
  // INC = 1: K-step of the next DMA issue as three digits, fastest first, advanced without
  // divisions: (s, r, cb) in the channel-block-major order (a.korder), (cb, s, r) in the tap-major one
  const bool ko = a.korder != 0;
  const int L0 = ko ? a.S : CB, L1 = ko ? a.R : a.S;
  int d0 = 0, d1 = 0, d2 = 0;
  auto advance = [&]() {
    d0 += 1;
    if (d0 == L0) {
      d0 = 0;
      d1 += 1;
      if (d1 == L1) {
        d1 = 0;
        d2 += 1;
      }
    }
  };
  auto issue_inc = [&](const Ctx& c, unsigned stage) {
    const int is = ko ? d0 : d1, ir = ko ? d1 : d2, icb = ko ? d2 : d0;
    const int rs = ir * a.S + is;
    char* As = smem + stage * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int q = 0; q < AI; ++q)
      lds_dma16s(c.wr, As + (wid * AI + q) * 1024, alane + (unsigned)((rs * CB + icb) * KB), aoff_s(q));
    const unsigned toff = (unsigned)((((ir - a.pad) * a.W + (is - a.pad)) * a.ldx + icb * 32) * 4);
    const unsigned need = tap_need(ir, is);
#pragma unroll
    for (int i = 0; i < BI; ++i)
      lds_dma16(c.xr, Bs + (wid * BI + i) * 1024,
                tapmask_ok<BI>(c.tm, i, need) ? c.bofs + cbytes[i] + (toff + (unsigned)(i * 8 * a.ldx * 4)) : 0xFFFFFFF0u);
    advance();
  };
  // SCH 5: the pieces of issue_inc's K-step into registers (ra: filter, rb: pixels), then stored to a stage
  u4v ra[RSTG ? AI : 1], rb[RSTG ? BI : 1];
  auto load_inc = [&](const Ctx& c) __attribute__((always_inline)) {
    if constexpr (RSTG) {
      const int is = ko ? d0 : d1, ir = ko ? d1 : d2, icb = ko ? d2 : d0;
      const int rs = ir * a.S + is;
#pragma unroll
      for (int q = 0; q < AI; ++q)
        ra[q] = __builtin_bit_cast(u4v, __builtin_amdgcn_raw_buffer_load_b128(
                                            c.wr, alane + (unsigned)((rs * CB + icb) * KB), aoff_s(q), 0));
      const unsigned toff = (unsigned)((((ir - a.pad) * a.W + (is - a.pad)) * a.ldx + icb * 32) * 4);
      const unsigned need = tap_need(ir, is);
#pragma unroll
      for (int i = 0; i < BI; ++i)
        rb[i] = bload(c.xr, tapmask_ok<BI>(c.tm, i, need) ? c.bofs + cbytes[i] + (toff + (unsigned)(i * 8 * a.ldx * 4))
                                                           : 0xFFFFFFF0u);
      advance();
    }
  };
  auto store_stage = [&](unsigned stage) __attribute__((always_inline)) {
    if constexpr (RSTG) {
      char* As = smem + stage * STAGE;
      char* Bs = As + A_BYTES;
#pragma unroll
      for (int q = 0; q < AI; ++q) *(u4v*)(As + (wid * AI + q) * 1024 + lane * 16) = ra[q];
#pragma unroll
      for (int i = 0; i < BI; ++i) *(u4v*)(Bs + (wid * BI + i) * 1024 + lane * 16) = rb[i];
    }
  };
  // SCH >= 1: piece p (< AI: filter, else pixels) of the DMA issue_inc makes; the caller advances the
  // cursor after the last piece
  auto issue_piece = [&](const Ctx& c, unsigned stage, int pc) __attribute__((always_inline)) {
    const int is = ko ? d0 : d1, ir = ko ? d1 : d2, icb = ko ? d2 : d0;
    const int rs = ir * a.S + is;
    char* As = smem + stage * STAGE;
    if (pc < AI) {
      lds_dma16s(c.wr, As + (wid * AI + pc) * 1024, alane + (unsigned)((rs * CB + icb) * KB), aoff_s(pc));
    } else {
      const int i = pc - AI;
      const unsigned toff = (unsigned)((((ir - a.pad) * a.W + (is - a.pad)) * a.ldx + icb * 32) * 4);
      lds_dma16(c.xr, As + A_BYTES + (wid * BI + i) * 1024,
                tapmask_ok<BI>(c.tm, i, tap_need(ir, is)) ? c.bofs + cbytes[i] + (toff + (unsigned)(i * 8 * a.ldx * 4))
                                                          : 0xFFFFFFF0u);
    }
  };
  auto issue = [&](const Ctx& c, int kt, int stage) {
    const int rs = a.korder ? kt % RS : kt / CB, cb = a.korder ? kt / RS : kt - rs * CB;
    const int r = rs / a.S, s2 = rs - r * a.S;
    char* As = smem + stage * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int q = 0; q < AI; ++q)
      lds_dma16s(c.wr, As + (wid * AI + q) * 1024, alane + (unsigned)((rs * CB + cb) * KB), aoff_s(q));
    const int dh = r - a.pad, dw = s2 - a.pad;
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int hh = c.pp[i] + dh, ww = c.pq[i] + dw;
      const bool ok = (unsigned)hh < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
      const unsigned off =
          ok ? (unsigned)(((long long)((c.prow0 + 8 * i) + dh * a.W + dw) * a.ldx + cb * 32) * 4) + cbytes[i] : 0xFFFFFFF0u;
      lds_dma16(c.xr, Bs + (wid * BI + i) * 1024, off);
    }
  };

  int lin = blockIdx.x;
  if (lin >= ntile) return;
  if (e3_lds) {
    for (int c = tid; c < a.Cout; c += 512) {
      ebias[c] = a.bias ? a.bias[c] : 0.f;
      escl[c] = a.escale[c];
      eshf[c] = a.eshift[c];
    }
  } else if (a.bias && !TALL) {
    for (int c = tid; c < a.Cout; c += 512) bbuf[c] = a.bias[c];
  }
  if (HM && !TALL)
    for (int c = tid; c < a.Cout; c += 512) ((unsigned*)hbuf)[c] = ((const unsigned*)htail)[c];
  Ctx cur, nxt;
  setup(lin, cur);
  bool has_next = lin + G < ntile;
  if (has_next) setup(lin + G, nxt);
  const int wpx = (wid % NPXG) * (PSB / NPXG), wco = (wid / NPXG) * (BN / NCOG);
  const int fr = lane & 15, fc = lane >> 4;
  unsigned gs = 0;
  if constexpr (RSTG) {  // K-step 0 into stage 0, K-step 1 into registers (KT >= 2, checked by the launcher)
    load_inc(cur);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    store_stage(0);
    load_inc(cur);
  } else if constexpr (INC) {
    issue_inc(cur, 0);
    if (PF > 1) issue_inc(cur, 1);
  } else {
    issue(cur, 0, 0);
    if (PF > 1) issue(cur, 1, 1);
  }
  bool first_tile = true;
  unsigned long long st_sum[5] = {0, 0, 0, 0, 0}, st_prev = 0, st_nk = 0, st_tiles = 0;
  auto stamp = [&]() __attribute__((always_inline)) -> unsigned long long {
    unsigned long long t = 0;
    if constexpr (STAMP) {
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    return t;
  };
  if constexpr (STAMP) st_prev = stamp();
  if constexpr (SCH == 2) {
    if (wid >= 4) __builtin_amdgcn_s_setprio(1);
  }
  while (true) {
    f4v acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
    if constexpr (STAMP) {  // epilogue of the previous tile (and the prologue before the first)
      const unsigned long long s = stamp();
      st_sum[4] += s - st_prev;
      st_prev = s;
      ++st_tiles;
    }
    if constexpr (SCH == 6) {
      // every wave runs the same K-step code (barrier, prologue, barrier, MFMA block); waves 4-7 pass
      // one extra barrier at the tile's start and waves 0-3 one at its end, so a wave's k-th barrier
      // meets its SIMD partner's (k-1)-th: one runs its prologue while the other runs its MFMA block
      const bool lead = wid < 4;
      const unsigned gb = gs;  // stage counter of this tile's K-step 0
      s8v bh6[TJ][NPL], ah6[NPL];
      auto aread6 = [&](const char* As, int i, s8v (&ah)[NPL]) __attribute__((always_inline)) {
        const int row = wco + 16 * i + fr;
        const int off = row * AROWB + ((fc ^ psw_a(row)) << 4);
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) ah[pl] = *(const s8v*)(As + pl * BN * AROWB + off);
      };
      // K-step t + 1's DMA (or the next tile's K-step 0) into the stage K-step t - 1 held: issued by
      // the leaders after their second barrier of K-step t and by the trailers after their first,
      // which is the same barrier instant; every wave waits for its own pieces one phase later,
      // ahead of the barrier behind which the leaders read them
      auto dma6 = [&](int t) __attribute__((always_inline)) {
        const int u = t + 1;
        if (u < KT) issue_inc(cur, (gb + u) % STG);
        else if (has_next) {
          d0 = d1 = d2 = 0;
          issue_inc(nxt, (gb + u) % STG);
        }
      };
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // K-step 0 (issued before the loop / in the last tile)
      if (!lead) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      for (int t = 0; t < KT; ++t) {
        const char* As = smem + ((gb + t) % STG) * STAGE;
        const char* Bs = As + A_BYTES;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (!lead) dma6(t);
        {  // prologue: K-step t's pixel fragments read and split, the first filter fragment read
          u4v b0[TJ], b1[TJ];
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            b0[j] = *(const u4v*)(Bs + swzb(wpx + 16 * j + fr, 2 * fc));
            b1[j] = *(const u4v*)(Bs + swzb(wpx + 16 * j + fr, 2 * fc + 1));
          }
          aread6(As, 0, ah6);
#pragma unroll
          for (int j = 0; j < TJ; ++j) split2h_8(b0[j], b1[j], hsx, bh6[j][0], bh6[j][1]);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (!lead) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (lead) dma6(t);
#pragma unroll
        for (int i = 0; i < TI; ++i) {  // MFMA block of K-step t
          s8v an[NPL];
          if (i + 1 < TI) aread6(As, i + 1, an);
          __builtin_amdgcn_s_setprio(1);
          constexpr int PA[3] = {1, 0, 0}, PB[3] = {0, 1, 0};
#pragma unroll
          for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, ah6[PA[q]]),
                                                                 __builtin_bit_cast(h8v, bh6[j][PB[q]]), acc[i][j], 0, 0, 0);
          __builtin_amdgcn_s_setprio(0);
          if (i + 1 < TI) {
#pragma unroll
            for (int pl = 0; pl < NPL; ++pl) ah6[pl] = an[pl];
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        if (lead) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if (lead) {  // meets the trailers' second barrier of the last K-step
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      gs = gb + KT;
    } else
    for (int t = 0; t < KT; ++t, ++gs) {
      const bool more = t + 1 < KT || has_next;
      if constexpr (RSTG) {  // the stage was written by ds_write: lgkmcnt below + the barrier order it
      } else if (PF > 1 && more && (t > 0 || first_tile)) {
        if constexpr (AI + BI == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
        else if constexpr (AI + BI == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      unsigned long long st_a = 0;
      if constexpr (STAMP) {
        st_a = stamp();
        st_sum[0] += st_a - st_prev;
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if constexpr (STAMP) {
        const unsigned long long s = stamp();
        st_sum[1] += s - st_a;
        st_a = s;
      }
      const char* As = smem + (gs % STG) * STAGE;
      const char* Bs = As + A_BYTES;
      if constexpr (SCH == 9) {  // this wave's half of its pixel group's rows into the SCH 8 image, in place
        char* Bw = smem + (gs % STG) * STAGE + A_BYTES;
        constexpr int ROWS = PSB / NPXG / NCOG;  // 32 rows: 4 lanes (8-channel groups) per row
        constexpr int NIT = ROWS * 4 / 64;
        const int r0 = wpx + ROWS * (wid / NPXG) + (lane >> 2), cj = lane & 3;
        u4v c0[NIT], c1[NIT];
#pragma unroll
        for (int k = 0; k < NIT; ++k) {
          c0[k] = *(const u4v*)(Bw + swzb(r0 + 16 * k, 2 * cj));
          c1[k] = *(const u4v*)(Bw + swzb(r0 + 16 * k, 2 * cj + 1));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < NIT; ++k) {
          s8v hi, lo;
          split2h_8(c0[k], c1[k], hsx, hi, lo);
          *(s8v*)(Bw + swzb(r0 + 16 * k, cj)) = hi;
          *(s8v*)(Bw + swzb(r0 + 16 * k, 4 + cj)) = lo;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      u4v b0[TJ], b1[TJ];
#pragma unroll
      for (int j = 0; j < TJ; ++j) {  // SCH 8 / 9: the hi / lo chunks of the pre-split rows, else two f32 chunks
        b0[j] = *(const u4v*)(Bs + swzb(wpx + 16 * j + fr, PRE ? fc : 2 * fc));
        b1[j] = *(const u4v*)(Bs + swzb(wpx + 16 * j + fr, PRE ? 4 + fc : 2 * fc + 1));
      }
      auto aread = [&](int i, s8v (&ah)[NPL]) __attribute__((always_inline)) {
        const int row = wco + 16 * i + fr;
        const int off = row * AROWB + ((fc ^ psw_a(row)) << 4);
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) ah[pl] = *(const s8v*)(As + pl * BN * AROWB + off);
      };
      s8v ah[NPL];
      aread(0, ah);
      // the next DMA: now (SCH 0), or one piece per MFMA block below (SCH >= 1)
      const int u_dma = t + PF;
      const bool dma_cur = u_dma < KT, dma_nxt = !dma_cur && has_next;
      if constexpr (RSTG) {
        // K-step u_dma (loaded a K-step ago) into its stage: every wave is past this K-step's barrier,
        // so done reading that stage (it held K-step t - 1); then K-step t + 2 into the registers
        if (dma_cur || dma_nxt) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          store_stage((gs + PF) % STG);
        }
        const int u2 = t + 2;
        if (u2 < KT) load_inc(cur);
        else if (has_next) {
          if (u2 == KT) d0 = d1 = d2 = 0;
          load_inc(nxt);
        }
      } else if constexpr (SCH == 3 || SCH == 4) {
        if (dma_nxt && u_dma == KT) d0 = d1 = d2 = 0;
        if (wid < 4) {
          if (dma_cur) issue_inc(cur, (gs + PF) % STG);
          else if (dma_nxt) issue_inc(nxt, (gs + PF) % STG);
        }
      } else if constexpr (SCH == 1 || SCH == 2) {
        if (dma_nxt && u_dma == KT) d0 = d1 = d2 = 0;
      } else {
        const int u = u_dma;
        if constexpr (INC) {
          if (u < KT) issue_inc(cur, (gs + PF) % STG);
          else if (has_next) {
            if (u == KT) d0 = d1 = d2 = 0;
            issue_inc(nxt, (gs + PF) % STG);
          }
        } else {
          if (u < KT) issue(cur, u, (gs + PF) % STG);
          else if (has_next) issue(nxt, u - KT, (gs + PF) % STG);
        }
      }
      s8v bh[TJ][NPL];
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        if constexpr (SCH == 7 || PRE) {  // 8 / 9: the parts as stored; 7 (diagnostic): the raw f32 rows
          bh[j][0] = __builtin_bit_cast(s8v, b0[j]);
          bh[j][1] = __builtin_bit_cast(s8v, b1[j]);
        } else if constexpr (HM) split2h_8(b0[j], b1[j], hsx, bh[j][0], bh[j][1]);
        else split3_8(b0[j], b1[j], bh[j][0], bh[j][1], bh[j][2]);
      }
      if constexpr (HM) __builtin_amdgcn_sched_barrier(0);  // the raw rows die here (else: 59 spilled VGPRs)
      if constexpr (STAMP) {
        const unsigned long long s = stamp();
        st_sum[2] += s - st_a;
        st_a = s;
      }
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        s8v an[NPL];
        if (i + 1 < TI) aread(i + 1, an);
        if constexpr (SCH == 1 || SCH == 2) {  // one DMA piece of the next K-step per MFMA block
          static_assert(SCH == 0 || AI + BI <= TI, "SCH: one piece per MFMA block");
          if (i < AI + BI) {
            if (dma_cur) issue_piece(cur, (gs + PF) % STG, i);
            else if (dma_nxt) issue_piece(nxt, (gs + PF) % STG, i);
            if (i == AI + BI - 1 && (dma_cur || dma_nxt)) advance();
          }
        }
        if constexpr (SCH != 2 && SCH != 4) __builtin_amdgcn_s_setprio(1);
        if constexpr (HM) {
          constexpr int PA[3] = {1, 0, 0}, PB[3] = {0, 1, 0};
#pragma unroll
          for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, ah[PA[q]]),
                                                                 __builtin_bit_cast(h8v, bh[j][PB[q]]), acc[i][j], 0, 0, 0);
        } else {
          constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
          for (int q = 0; q < 6; ++q)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[PA[q]], bh[j][PB[q]], acc[i][j], 0, 0, 0);
        }
        if constexpr (SCH != 2 && SCH != 4) __builtin_amdgcn_s_setprio(0);
        if (i + 1 < TI) {
#pragma unroll
          for (int pl = 0; pl < NPL; ++pl) ah[pl] = an[pl];
        }
        if constexpr (HM) __builtin_amdgcn_sched_barrier(0);  // no fragment reads hoisted across blocks
      }
      if constexpr (SCH == 3 || SCH == 4) {  // waves 4-7: the next K-step's DMA after their MFMA block
        if (wid >= 4) {
          if (dma_cur) issue_inc(cur, (gs + PF) % STG);
          else if (dma_nxt) issue_inc(nxt, (gs + PF) % STG);
        }
      }
      if constexpr (STAMP) {
        st_prev = stamp();
        st_sum[3] += st_prev - st_a;
        ++st_nk;
      }
    }
    first_tile = false;
    if constexpr (TALL) {  // the consumed stage becomes the epilogue scratch: this tile's bias, statistics
      epi_lds = smem + ((gs - 1) % STG) * STAGE;
      bbuf = (float*)(epi_lds + EPI_B) - cur.co0;  // indexed by absolute channel
      lds_barrier();  // every wave is done reading the stage
      if (a.bias && tid < BN) bbuf[cur.co0 + tid] = a.bias[cur.co0 + tid];
      hbuf = bbuf + BN;  // absolute channel index, as bbuf
      if (HM && tid < BN) ((unsigned*)hbuf)[cur.co0 + tid] = ((const unsigned*)htail)[cur.co0 + tid];
      lds_barrier();
    }
    // HM: back from the scaled operands, exact powers of two per output channel, applied where the
    // epilogue first reads acc (a separate pass over all of acc ahead of the stores spilled 59 VGPRs)
    auto hscale = [&](int i, int j) __attribute__((always_inline)) {
      if constexpr (HM) {  // the tail words hold the exponents (split_weight_h_kernel)
        const u4v sc = *(const u4v*)(hbuf + cur.co0 + wco + 16 * i + 4 * fc);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = ldexpf(acc[i][j][r], (int)sc[r]);
      }
    };
    float* y = (float*)a.y;
    bool valid[TJ];
    // y += old y ahead of the stores (EPI_ACC_NOTE)
    if (a.accumulate) {
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int px = cur.px0 + wpx + 16 * j + fr;
        if (px >= M) continue;
        const float* yrow = y + (long long)px * a.ldy;
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int co = cur.co0 + wco + 16 * i + 4 * fc;
          hscale(i, j);
          if (e3_lds) {
            const f4v b = *(const f4v*)(ebias + co);
            for (int r = 0; r < 4; ++r) acc[i][j][r] += b[r];
          } else if (a.bias) {
            const f4v b = *(const f4v*)(bbuf + co);
            for (int r = 0; r < 4; ++r) acc[i][j][r] += b[r];
          }
          add_old_y(acc[i][j], yrow, a, px, co);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int px = cur.px0 + wpx + 16 * j + fr;
      valid[j] = px < M;
      if (px >= M) continue;
      float* yrow = y + (long long)px * a.ldy;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int co = cur.co0 + wco + 16 * i + 4 * fc;
        if (!a.accumulate) hscale(i, j);
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if (a.accumulate) {
        } else if (e3_lds) {
          const f4v b = *(const f4v*)(ebias + co);
          v[0] += b[0]; v[1] += b[1]; v[2] += b[2]; v[3] += b[3];
        } else if (a.bias) {
          const f4v b = *(const f4v*)(bbuf + co);
          v[0] += b[0]; v[1] += b[1]; v[2] += b[2]; v[3] += b[3];
        }
        if constexpr (EPI == 3) {
          if (e3_lds) {  // same fmaf / ReLU as epi_affine on the same f32 value
            const f4v sc = *(const f4v*)(escl + co), sf = *(const f4v*)(eshf + co);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float tt = fmaf(v[r], sc[r], sf[r]);
              if (a.eact == 1) tt = tt > 0.f ? tt : 0.f;
              v[r] = tt;
            }
          } else {
            epi_affine(v, a, co);
          }
        }
        st4(yrow + co, v);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = v[r];
      }
    }
    if constexpr (EPI == 2)  // dgrad: BatchNorm-backward partials of the layer whose gradient this is
      epi_bnbwd<TI, TJ, NPXG, BN, float, PSB>(acc, valid, wid % NPXG, wco, wpx, epi_lds, a, cur.px0, cur.co0, tid, fr,
                                             fc);
    if (EPI == 0 && a.part)
      epi_stats<TI, TJ, NPXG, BN>(acc, valid, wid % NPXG, wco, epi_lds, a.part + (long long)(cur.px0 / PSB) * 3 * a.Cout,
                               a.Cout, cur.co0, tid, fr, fc);
    if (!has_next) break;
    cur = nxt;
    lin += G;
    has_next = lin + G < ntile;
    if (has_next) setup(lin + G, nxt);
  }
  if constexpr (STAMP) {  // the last tile's epilogue, then one row of 8 per wave
    st_sum[4] += stamp() - st_prev;
    if (lane == 0 && a.stamps) {
      unsigned long long* o = a.stamps + ((long long)blockIdx.x * 8 + wid) * 8;
      for (int q = 0; q < 5; ++q) o[q] = st_sum[q];
      o[5] = st_nk;
      o[6] = st_tiles;
      o[7] = (unsigned long long)KT;
    }
  }
}

// f32 forward/dgrad for Cout = 64 layers on the split math, both operands split ONCE per
// block: the pre-split filter planes (split_weight_kernel) and the f32 pixel rows are loaded
// to registers one K-step ahead; the pixel rows are split while being stored to LDS as three
// bf16 planes (64-B rows, chunk c of row r at c ^ psw_a(r), as the filter planes).
// Tile 64 channels x 256 pixels, 8 waves of 64 pixels x 32 channels, 32-channel K-steps,
// double-buffered LDS (2 x 60 KB).  With only two channel fragments per wave, the per-wave
// pixel split of conv_fwd_pers_kernel<64, .., SPL = 1> cost more VALU than its MFMAs.
// HM = 1: the f16 x3 arithmetic (two f16 planes per operand: presplit_h's filter planes and scales, the
// pixel rows scaled by the tensor's power of two), three f16 MFMAs per block.
template <int EPI = 0, int HM = 0>
__global__ __launch_bounds__(512, 1) void conv_fwd_rsplit_kernel(FwdArgs a, const char* __restrict__ wsp) {
  constexpr int BN = 64, BPX = 256;
  constexpr int NPL = HM ? 2 : 3, KB = NPL * 64;  // planes; bytes per (co, k-block) of the filter planes
  constexpr int A_PL = BN * 64, B_PL = BPX * 64;  // plane bytes
  constexpr int BUF = NPL * (A_PL + B_PL);
  constexpr int TI = 2, TJ = 4;
  constexpr int BR = BPX * 8 / 512;               // 16-B f32 chunks of the pixel tile per thread
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  const int HW = a.H * a.W;
  const int M = a.N * HW;
  const int nco = a.Cout / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int co0 = (bid % nco) * BN;
  const int px0 = (bid / nco) * BPX;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int chunk = tid & 7, rbase = tid >> 3;
  const int CB = a.C / 32;
  const int KT = a.R * a.S * CB;

  const int halo = a.pad * (a.W + 1);
  const int plo = max(0, px0 - halo);
  const int phi = min(M, px0 + BPX + halo);
  const unsigned win_bytes = (unsigned)(((long long)(phi - plo - 1) * a.ldx + a.C) * 4);
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.x + (long long)plo * a.ldx * 4), 0,
                                                                win_bytes, 0x00020000);
  int pp[BR], pq[BR], prow[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int m = px0 + rbase + 64 * i;
    const int rem = m % HW;
    prow[i] = m;
    pp[i] = (m < M) ? rem / a.W : -100000;
    pq[i] = rem % a.W;
  }
  // filter-plane chunks: q = tid (all threads) and q = tid + 512 (tid < 256, three planes only);
  // q -> (plane, row, chunk)
  const char* wbase = wsp + (long long)co0 * KT * KB;
  auto wq_off = [&](int q) { return (long long)((q & 255) >> 2) * KT * KB + (q >> 8) * 64 + (q & 3) * 16; };
  auto wq_lds = [&](int q) {
    const int row = (q & 255) >> 2;
    return (q >> 8) * A_PL + row * 64 + (((q & 3) ^ psw_a(row)) << 4);
  };
  const long long wo0 = wq_off(tid), wo1 = wq_off(tid + 512);
  const int wl0 = wq_lds(tid), wl1 = wq_lds(tid + 512);
  // HM: the scales after the planes ([Cout] the rescale exponents -(e_row + e_x) as int bits, then s_x)
  const float* htail = (const float*)(wsp + (long long)a.Cout * KT * KB);
  const float hsx = HM ? htail[a.Cout] : 1.f;

  u4v ra0, ra1, rb[BR];
  auto gload = [&](int t) __attribute__((always_inline)) {
    const int rs = t / CB, cb = t - rs * CB;
    const int r = rs / a.S, s2 = rs - r * a.S;
    ra0 = *(const u4v*)(wbase + wo0 + (long long)t * KB);
    if (!HM && tid < 256) ra1 = *(const u4v*)(wbase + wo1 + (long long)t * KB);
    const int dh = r - a.pad, dw = s2 - a.pad;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int h = pp[i] + dh, ww = pq[i] + dw;
      const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
      const long long pin = (long long)(prow[i] + dh * a.W + dw - plo);
      const unsigned off = ok ? (unsigned)((pin * a.ldx + cb * 32 + chunk * 4) * 4) : 0xFFFFFFF0u;
      rb[i] = bload(xr, off);
    }
  };
  auto swrite = [&](int buf) __attribute__((always_inline)) {
    char* As = smem + buf * BUF;
    char* Bs = As + NPL * A_PL;
    *(u4v*)(As + wl0) = ra0;
    if (!HM && tid < 256) *(u4v*)(As + wl1) = ra1;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int row = rbase + 64 * i;
      const int o = row * 64 + ((((chunk >> 1) ^ psw_a(row))) << 4) + (chunk & 1) * 8;
      if constexpr (HM) {
        u2v h0, h1;
        split2h_4(rb[i], hsx, h0, h1);
        *(u2v*)(Bs + o) = h0;
        *(u2v*)(Bs + B_PL + o) = h1;
      } else {
        u2v h0, h1, h2;
        split3_4(rb[i], h0, h1, h2);
        *(u2v*)(Bs + o) = h0;
        *(u2v*)(Bs + B_PL + o) = h1;
        *(u2v*)(Bs + 2 * B_PL + o) = h2;
      }
    }
  };

  f4v acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  const int wpx = (wid & 3) * 64, wco = (wid >> 2) * 32;
  const int fr = lane & 15, fc = lane >> 4;

  gload(0);
  swrite(0);
  __syncthreads();
  for (int t = 0; t < KT; ++t) {
    const int cur = t & 1;
    if (t + 1 < KT) gload(t + 1);
    const char* As = smem + cur * BUF;
    const char* Bs = As + NPL * A_PL;
    s8v bh[TJ][NPL], ah[TI][NPL];
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int row = wpx + 16 * j + fr;
      const int o = row * 64 + ((fc ^ psw_a(row)) << 4);
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) bh[j][pl] = *(const s8v*)(Bs + pl * B_PL + o);
    }
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int row = wco + 16 * i + fr;
      const int o = row * 64 + ((fc ^ psw_a(row)) << 4);
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) ah[i][pl] = *(const s8v*)(As + pl * A_PL + o);
    }
    if constexpr (HM) {
      constexpr int PA3[3] = {1, 0, 0}, PB3[3] = {0, 1, 0};
#pragma unroll
      for (int u = 0; u < 3; ++u) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, ah[i][PA3[u]]),
                                                               __builtin_bit_cast(h8v, bh[j][PB3[u]]), acc[i][j], 0, 0, 0);
        if (u == 1 && t + 1 < KT) swrite(cur ^ 1);  // overlapped with the remaining products
      }
    } else {
      constexpr int PA6[6] = {2, 1, 0, 1, 0, 0}, PB6[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
      for (int u = 0; u < 6; ++u) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i][PA6[u]], bh[j][PB6[u]], acc[i][j], 0, 0, 0);
        if (u == 2 && t + 1 < KT) swrite(cur ^ 1);  // overlapped with the remaining products
      }
    }
    __syncthreads();
  }
  if constexpr (HM) {  // back from the scaled operands (exact powers of two per output channel)
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const u4v sc = *(const u4v*)(htail + co0 + wco + 16 * i + 4 * fc);  // exponents (split_weight_h_kernel)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = ldexpf(acc[i][j][r], (int)sc[r]);
    }
  }

  float* y = (float*)a.y;
  bool valid[TJ];
  f4v bv[TI];  // bias read once, ahead of the stores (EPI_ACC_NOTE)
#pragma unroll
  for (int i = 0; i < TI; ++i)
    bv[i] = a.bias ? *(const f4v*)(a.bias + co0 + wco + 16 * i + 4 * fc) : f4v{0.f, 0.f, 0.f, 0.f};
  if (a.accumulate || EPI == 3) {  // old y, bias and the eval-BN affine ahead of the stores (EPI_ACC_NOTE)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int px = px0 + wpx + 16 * j + fr;
      if (px >= M) continue;
      const float* yrow = y + (long long)px * a.ldy;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int co = co0 + wco + 16 * i + 4 * fc;
        if (a.bias) {
          const f4v b = *(const f4v*)(a.bias + co);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += b[r];
        }
        if (a.accumulate) add_old_y(acc[i][j], yrow, a, px, co);
        if constexpr (EPI == 3) {
          float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
          epi_affine(v, a, co);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = v[r];
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int px = px0 + wpx + 16 * j + fr;
    valid[j] = px < M;
    if (px >= M) continue;
    float* yrow = y + (long long)px * a.ldy;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int co = co0 + wco + 16 * i + 4 * fc;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (a.bias && !a.accumulate && EPI != 3) {
        const f4v b = bv[i];
        v[0] += b[0]; v[1] += b[1]; v[2] += b[2]; v[3] += b[3];
      }
      st4(yrow + co, v);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = v[r];
    }
  }
  if (EPI == 0 && a.part)  // smem reuse: every wave is past the K loop's last barrier
    epi_stats<TI, TJ, 4, BN>(acc, valid, wid & 3, wco, smem, a.part + (long long)(px0 / BPX) * 3 * a.Cout, a.Cout,
                             co0, tid, fr, fc);
}

// conv_fwd_rsplit_kernel with the three taps of a kernel row sharing one staged pixel strip
// (3x3 / pad 1, W % 256 == 0, so a 256-pixel tile is one image-row segment): a K-step is
// (kernel row r, 32-channel block); the strip X[258 px][32 c] of image row p + r - 1 (columns
// q0 - 1 .. q0 + 256) is loaded, split ONCE into three bf16 planes and read by the taps
// s = 0, 1, 2 at row offsets s, so the split and LDS-store work per MFMA is 1/3 of the per-tap
// kernel's.  The three taps' pre-split filter planes (36 KB) are staged through registers into a
// single LDS buffer (two barriers per K-step: the strip takes the double buffer); reading them
// per wave straight from L2 measured no faster than the per-tap kernel (8 waves x 18 KB per
// K-step per CU of L2 traffic).  Same tile (256 px x 64 co, 8 waves of 64 px x 32 co) and
// epilogues as conv_fwd_rsplit_kernel; K order (r, c-block, s) instead of (r, s, c-block).
// HM = 1: the f16 x3 arithmetic (two f16 planes per operand, presplit_h's filter planes and scales).
template <int EPI = 0, int HM = 0>
__global__ __launch_bounds__(512, 1) void conv_fwd_rsplit3_kernel(FwdArgs a, const char* __restrict__ wsp) {
  constexpr int NPL = HM ? 2 : 3, KB = NPL * 64;       // planes; bytes per (co, k-block) of the filter planes
  constexpr int BN = 64, BPX = 256, SR = 264;        // strip rows (258 used)
  constexpr int B_PL = SR * 64, BUF = NPL * B_PL;    // strip plane / buffer bytes
  constexpr int A_PL = BN * 64, A_TAP = NPL * A_PL;  // filter plane / tap bytes
  constexpr int TI = 2, TJ = 4;
  constexpr int NCH = (BPX + 2) * 8, BR = (NCH + 511) / 512;  // 16-B f32 chunks of the strip
  constexpr int NA = 3 * NPL * BN * 4, AR = (NA + 511) / 512;  // 16-B chunks of the 3 taps' planes
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF + 3 * A_TAP];
  char* Asm = smem + 2 * BUF;

  const int HW = a.H * a.W;
  const int M = a.N * HW;
  const int nco = a.Cout / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int co0 = (bid % nco) * BN;
  const int px0 = (bid / nco) * BPX;
  const int tn = px0 / HW, tp = (px0 - tn * HW) / a.W, tq = px0 - tn * HW - tp * a.W;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int chunk = tid & 7, rbase = tid >> 3;
  const int CB = a.C / 32;
  const int KT3 = 3 * CB;

  const int plo = max(0, px0 - (a.W + 1));
  const int phi = min(M, px0 + BPX + a.W + 1);
  const unsigned win_bytes = (unsigned)(((long long)(phi - plo - 1) * a.ldx + a.C) * 4);
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.x + (long long)plo * a.ldx * 4), 0,
                                                                win_bytes, 0x00020000);
  const int wpx = (wid & 3) * 64, wco = (wid >> 2) * 32;
  const int fr = lane & 15, fc = lane >> 4;
  // filter chunk q of a K-step: (tap s, plane, row co, 16-B chunk) = (q / (NPL 256), (q / 256) % NPL, (q & 255) >> 2, q & 3)
  const char* wbase = wsp + (long long)co0 * (9 * CB) * KB;
  int a_src[AR], a_dst[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int q = tid + 512 * i;
    const int ts = q / (NPL * 256), pl = (q / 256) % NPL, row = (q & 255) >> 2, ch = q & 3;
    a_src[i] = q < NA ? (row * (9 * CB) + ts * CB) * KB + pl * 64 + ch * 16 : -1;  // + (r*3*CB + cb)*KB
    a_dst[i] = ts * A_TAP + pl * A_PL + row * 64 + ((ch ^ psw_a(row)) << 4);
  }
  // HM: the scales after the planes ([Cout] the rescale exponents -(e_row + e_x) as int bits, then s_x)
  const float* htail = (const float*)(wsp + (long long)a.Cout * 9 * CB * KB);
  const float hsx = HM ? htail[a.Cout] : 1.f;

  u4v rb[BR], ra[AR];
  auto gload = [&](int t) __attribute__((always_inline)) {
    const int r = t / CB, cb = t - r * CB;
    const int h = tp + r - 1;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int row = rbase + 64 * i;
      const int ww = tq - 1 + row;
      const bool ok = row < BPX + 2 && (unsigned)h < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
      const long long pin = (long long)tn * HW + (long long)h * a.W + ww - plo;
      rb[i] = bload(xr, ok ? (unsigned)((pin * a.ldx + cb * 32 + chunk * 4) * 4) : 0xFFFFFFF0u);
    }
    const long long koff = (long long)(r * 3 * CB + cb) * KB;
#pragma unroll
    for (int i = 0; i < AR; ++i)
      if (a_src[i] >= 0) ra[i] = *(const u4v*)(wbase + a_src[i] + koff);
  };
  auto swrite = [&](int buf) __attribute__((always_inline)) {
    char* Bs = smem + buf * BUF;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int row = rbase + 64 * i;
      if (row < BPX + 2) {
        const int o = row * 64 + ((((chunk >> 1) ^ psw_a(row))) << 4) + (chunk & 1) * 8;
        if constexpr (HM) {
          u2v h0, h1;
          split2h_4(rb[i], hsx, h0, h1);
          *(u2v*)(Bs + o) = h0;
          *(u2v*)(Bs + B_PL + o) = h1;
        } else {
          u2v h0, h1, h2;
          split3_4(rb[i], h0, h1, h2);
          *(u2v*)(Bs + o) = h0;
          *(u2v*)(Bs + B_PL + o) = h1;
          *(u2v*)(Bs + 2 * B_PL + o) = h2;
        }
      }
    }
  };

  f4v acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  gload(0);
  swrite(0);
  for (int t = 0; t < KT3; ++t) {
    const int cur = t & 1;
    __syncthreads();  // every wave is done with the previous K-step's filter planes
#pragma unroll
    for (int i = 0; i < AR; ++i)
      if (a_src[i] >= 0) *(u4v*)(Asm + a_dst[i]) = ra[i];
    __syncthreads();  // filter planes of this K-step (and its strip, stored during the last one) visible
    if (t + 1 < KT3) gload(t + 1);
    const char* Bs = smem + cur * BUF;
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      s8v ah[TI][NPL], bh[TJ][NPL];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int row = wco + 16 * i + fr;
        const int o = s * A_TAP + row * 64 + ((fc ^ psw_a(row)) << 4);
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) ah[i][pl] = *(const s8v*)(Asm + pl * A_PL + o);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int row = wpx + 16 * j + fr + s;
        const int o = row * 64 + ((fc ^ psw_a(row)) << 4);
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) bh[j][pl] = *(const s8v*)(Bs + pl * B_PL + o);
      }
      if constexpr (HM) {
        constexpr int PA3[3] = {1, 0, 0}, PB3[3] = {0, 1, 0};
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, ah[i][PA3[u]]),
                                                                 __builtin_bit_cast(h8v, bh[j][PB3[u]]), acc[i][j], 0, 0, 0);
      } else {
        constexpr int PA6[6] = {2, 1, 0, 1, 0, 0}, PB6[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
        for (int u = 0; u < 6; ++u)
#pragma unroll
          for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i][PA6[u]], bh[j][PB6[u]], acc[i][j], 0, 0, 0);
      }
      if (s == 1 && t + 1 < KT3) swrite(cur ^ 1);  // the other buffer was last read before this step's barriers
    }
  }
  __syncthreads();  // smem reuse by the statistics epilogue
  if constexpr (HM) {  // back from the scaled operands (exact powers of two per output channel)
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const u4v sc = *(const u4v*)(htail + co0 + wco + 16 * i + 4 * fc);  // exponents (split_weight_h_kernel)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = ldexpf(acc[i][j][r], (int)sc[r]);
    }
  }

  float* y = (float*)a.y;
  bool valid[TJ];
  f4v bv[TI];  // bias read once, ahead of the stores (EPI_ACC_NOTE)
#pragma unroll
  for (int i = 0; i < TI; ++i)
    bv[i] = a.bias ? *(const f4v*)(a.bias + co0 + wco + 16 * i + 4 * fc) : f4v{0.f, 0.f, 0.f, 0.f};
  if (a.accumulate || EPI == 3) {  // old y, bias and the eval-BN affine ahead of the stores (EPI_ACC_NOTE)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int px = px0 + wpx + 16 * j + fr;
      if (px >= M) continue;
      const float* yrow = y + (long long)px * a.ldy;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int co = co0 + wco + 16 * i + 4 * fc;
        if (a.bias) {
          const f4v b = *(const f4v*)(a.bias + co);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += b[r];
        }
        if (a.accumulate) add_old_y(acc[i][j], yrow, a, px, co);
        if constexpr (EPI == 3) {
          float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
          epi_affine(v, a, co);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = v[r];
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int px = px0 + wpx + 16 * j + fr;
    valid[j] = px < M;
    if (px >= M) continue;
    float* yrow = y + (long long)px * a.ldy;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int co = co0 + wco + 16 * i + 4 * fc;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (a.bias && !a.accumulate && EPI != 3) {
        const f4v b = bv[i];
        v[0] += b[0]; v[1] += b[1]; v[2] += b[2]; v[3] += b[3];
      }
      st4(yrow + co, v);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = v[r];
    }
  }
  if (EPI == 0 && a.part)
    epi_stats<TI, TJ, 4, BN>(acc, valid, wid & 3, wco, smem, a.part + (long long)(px0 / BPX) * 3 * a.Cout, a.Cout,
                             co0, tid, fr, fc);
}

// conv_fwd_rsplit3_kernel on 512-pixel tiles (W % 512 == 0) with all 8 waves on pixels, each
// 64 channels x 64 pixels (twice the per-wave fragment reuse of the 2 x 4 layout): the 514-pixel
// strip (99 KB of planes) and the three taps' filter planes (36 KB) are single-buffered, both
// stored between the K-step's two barriers from registers loaded during the previous K-step.
// HM = 1: the f16 x3 arithmetic (two f16 planes per operand, presplit_h's filter planes and scales).
template <int EPI = 0, int HM = 0>
__global__ __launch_bounds__(512, 1) void conv_fwd_rsplit3w_kernel(FwdArgs a, const char* __restrict__ wsp) {
  constexpr int NPL = HM ? 2 : 3, KB = NPL * 64;        // planes; bytes per (co, k-block) of the filter planes
  constexpr int BN = 64, BPX = 512, SR = 520;        // strip rows (514 used)
  constexpr int B_PL = SR * 64, BUF = NPL * B_PL;    // strip plane / buffer bytes
  constexpr int A_PL = BN * 64, A_TAP = NPL * A_PL;  // filter plane / tap bytes
  constexpr int TI = 4, TJ = 4;
  constexpr int NCH = (BPX + 2) * 8, BR = (NCH + 511) / 512;  // 16-B f32 chunks of the strip
  constexpr int NA = 3 * NPL * BN * 4, AR = (NA + 511) / 512;  // 16-B chunks of the 3 taps' planes
  __shared__ __attribute__((aligned(16))) char smem[BUF + 3 * A_TAP];
  char* Asm = smem + BUF;

  const int HW = a.H * a.W;
  const int M = a.N * HW;
  const int nco = a.Cout / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int co0 = (bid % nco) * BN;
  const int px0 = (bid / nco) * BPX;
  const int tn = px0 / HW, tp = (px0 - tn * HW) / a.W, tq = px0 - tn * HW - tp * a.W;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int chunk = tid & 7, rbase = tid >> 3;
  const int CB = a.C / 32;
  const int KT3 = 3 * CB;

  const int plo = max(0, px0 - (a.W + 1));
  const int phi = min(M, px0 + BPX + a.W + 1);
  const unsigned win_bytes = (unsigned)(((long long)(phi - plo - 1) * a.ldx + a.C) * 4);
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.x + (long long)plo * a.ldx * 4), 0,
                                                                win_bytes, 0x00020000);
  const int wpx = wid * 64, wco = 0;
  const int fr = lane & 15, fc = lane >> 4;
  // filter chunk q of a K-step: (tap s, plane, row co, 16-B chunk) = (q / (NPL 256), (q / 256) % NPL, (q & 255) >> 2, q & 3)
  const char* wbase = wsp + (long long)co0 * (9 * CB) * KB;
  int a_src[AR], a_dst[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int q = tid + 512 * i;
    const int ts = q / (NPL * 256), pl = (q / 256) % NPL, row = (q & 255) >> 2, ch = q & 3;
    a_src[i] = q < NA ? (row * (9 * CB) + ts * CB) * KB + pl * 64 + ch * 16 : -1;  // + (r*3*CB + cb)*KB
    a_dst[i] = ts * A_TAP + pl * A_PL + row * 64 + ((ch ^ psw_a(row)) << 4);
  }
  // HM: the scales after the planes ([Cout] the rescale exponents -(e_row + e_x) as int bits, then s_x)
  const float* htail = (const float*)(wsp + (long long)a.Cout * 9 * CB * KB);
  const float hsx = HM ? htail[a.Cout] : 1.f;

  u4v rb[BR], ra[AR];
  auto gload = [&](int t) __attribute__((always_inline)) {
    const int r = t / CB, cb = t - r * CB;
    const int h = tp + r - 1;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int row = rbase + 64 * i;
      const int ww = tq - 1 + row;
      const bool ok = row < BPX + 2 && (unsigned)h < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
      const long long pin = (long long)tn * HW + (long long)h * a.W + ww - plo;
      rb[i] = bload(xr, ok ? (unsigned)((pin * a.ldx + cb * 32 + chunk * 4) * 4) : 0xFFFFFFF0u);
    }
    const long long koff = (long long)(r * 3 * CB + cb) * KB;
#pragma unroll
    for (int i = 0; i < AR; ++i)
      if (a_src[i] >= 0) ra[i] = *(const u4v*)(wbase + a_src[i] + koff);
  };
  auto swrite = [&](int buf) __attribute__((always_inline)) {
    char* Bs = smem + buf * 0;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int row = rbase + 64 * i;
      if (row < BPX + 2) {
        const int o = row * 64 + ((((chunk >> 1) ^ psw_a(row))) << 4) + (chunk & 1) * 8;
        if constexpr (HM) {
          u2v h0, h1;
          split2h_4(rb[i], hsx, h0, h1);
          *(u2v*)(Bs + o) = h0;
          *(u2v*)(Bs + B_PL + o) = h1;
        } else {
          u2v h0, h1, h2;
          split3_4(rb[i], h0, h1, h2);
          *(u2v*)(Bs + o) = h0;
          *(u2v*)(Bs + B_PL + o) = h1;
          *(u2v*)(Bs + 2 * B_PL + o) = h2;
        }
      }
    }
  };

  f4v acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  gload(0);
  for (int t = 0; t < KT3; ++t) {
    __syncthreads();  // every wave is done with the previous K-step's strip and filter planes
    swrite(0);
#pragma unroll
    for (int i = 0; i < AR; ++i)
      if (a_src[i] >= 0) *(u4v*)(Asm + a_dst[i]) = ra[i];
    __syncthreads();
    if (t + 1 < KT3) gload(t + 1);
    const char* Bs = smem;
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      s8v ah[TI][NPL], bh[TJ][NPL];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int row = wco + 16 * i + fr;
        const int o = s * A_TAP + row * 64 + ((fc ^ psw_a(row)) << 4);
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) ah[i][pl] = *(const s8v*)(Asm + pl * A_PL + o);
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int row = wpx + 16 * j + fr + s;
        const int o = row * 64 + ((fc ^ psw_a(row)) << 4);
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) bh[j][pl] = *(const s8v*)(Bs + pl * B_PL + o);
      }
      if constexpr (HM) {
        constexpr int PA3[3] = {1, 0, 0}, PB3[3] = {0, 1, 0};
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, ah[i][PA3[u]]),
                                                                 __builtin_bit_cast(h8v, bh[j][PB3[u]]), acc[i][j], 0, 0, 0);
      } else {
        constexpr int PA6[6] = {2, 1, 0, 1, 0, 0}, PB6[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
        for (int u = 0; u < 6; ++u)
#pragma unroll
          for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i][PA6[u]], bh[j][PB6[u]], acc[i][j], 0, 0, 0);
      }
    }
  }
  __syncthreads();  // smem reuse by the statistics epilogue

  float* y = (float*)a.y;
  bool valid[TJ];
  f4v bv[TI];  // bias read once, ahead of the stores (EPI_ACC_NOTE)
#pragma unroll
  for (int i = 0; i < TI; ++i)
    bv[i] = a.bias ? *(const f4v*)(a.bias + co0 + wco + 16 * i + 4 * fc) : f4v{0.f, 0.f, 0.f, 0.f};
  if constexpr (HM) {  // back from the scaled operands (exact powers of two per output channel)
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const u4v sc = *(const u4v*)(htail + co0 + wco + 16 * i + 4 * fc);  // exponents (split_weight_h_kernel)
#pragma unroll
      for (int j = 0; j < TJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = ldexpf(acc[i][j][r], (int)sc[r]);
    }
  }
  if (a.accumulate || EPI == 3) {  // old y, bias and the eval-BN affine ahead of the stores (EPI_ACC_NOTE)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int px = px0 + wpx + 16 * j + fr;
      if (px >= M) continue;
      const float* yrow = y + (long long)px * a.ldy;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int co = co0 + wco + 16 * i + 4 * fc;
        if (a.bias) {
          const f4v b = *(const f4v*)(a.bias + co);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] += b[r];
        }
        if (a.accumulate) add_old_y(acc[i][j], yrow, a, px, co);
        if constexpr (EPI == 3) {
          float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
          epi_affine(v, a, co);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = v[r];
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int px = px0 + wpx + 16 * j + fr;
    valid[j] = px < M;
    if (px >= M) continue;
    float* yrow = y + (long long)px * a.ldy;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int co = co0 + wco + 16 * i + 4 * fc;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (a.bias && !a.accumulate && EPI != 3) {
        const f4v b = bv[i];
        v[0] += b[0]; v[1] += b[1]; v[2] += b[2]; v[3] += b[3];
      }
      st4(yrow + co, v);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = v[r];
    }
  }
  if (EPI == 0 && a.part)
    epi_stats<TI, TJ, 8, BN>(acc, valid, wid, wco, smem, a.part + (long long)(px0 / BPX) * 3 * a.Cout, a.Cout,
                             co0, tid, fr, fc);
}

// wsp[co][kb][part][32] (bf16) = the exact 3-way split (dg_common.h split3_pair, truncated parts
// as the forward's pixel fragments) of the packed f32 filter w[co][kb*32 + j]; two elements per thread
__global__ void split_weight_kernel(const float* __restrict__ w, long long n, unsigned short* __restrict__ wsp) {
  const long long n2 = n >> 1;  // n = Cout*R*S*C is a multiple of 32
  for (long long o = blockIdx.x * (long long)blockDim.x + threadIdx.x; o < n2; o += (long long)gridDim.x * blockDim.x) {
    const float2 v = *(const float2*)(w + 2 * o);
    unsigned p0, p1, p2;
    split3_pair<false>(__float_as_uint(v.x), __float_as_uint(v.y), p0, p1, p2);
    const long long e = 2 * o, blk = e >> 5, j = e & 31;
    unsigned* d = (unsigned*)(wsp + blk * 96 + j);
    d[0] = p0;
    d[16] = p1;
    d[32] = p2;
  }
}

// f16 x3 filter planes (dg_common.h split2h_pair): one block per output row co of the packed
// f32 filter w[co][K]: the row's largest magnitude sets its power-of-two scale s_row, the parts of
// w * s_row go to wsp[co][kb][2][32] (f16 hi, lo), and after the Cout * K * 4 bytes of planes the
// tail [Cout] = 2^-(e_row + e_x) (the epilogue's exact rescale) and [Cout] = s_x = 2^e_x, from the
// pixel operand's largest magnitude *xamax (amax_kernel).  The rescale is stored as the integer exponent
// -(e_row + e_x) in the float word's bits and applied with ldexp (exact whenever the result is an f32:
// a factor 2^-(e_row + e_x) itself leaves f32's range once both operands are tiny).
__global__ __launch_bounds__(256) void split_weight_h_kernel(const float* __restrict__ w, int K,
                                                           unsigned short* __restrict__ wsp,
                                                           const unsigned* __restrict__ xamax, int Cout) {
  __shared__ float red[4];
  const int co = blockIdx.x, tid = threadIdx.x;
  const float* row = w + (long long)co * K;
  float m = 0.f;
  for (int e = tid; e < K; e += 256) m = fmaxf(m, fabsf(row[e]));
  m = wave_max(m);
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const int er = h16_exp(m), ex = h16_exp(__uint_as_float(*xamax));
  const float s = ldexpf(1.f, er);
  for (int e = 2 * tid; e < K; e += 512) {
    unsigned ph, pl;
    split2h_pair(row[e], row[e + 1], s, ph, pl);
    unsigned* d = (unsigned*)(wsp + (((long long)co * K + e) >> 5) * 64 + (e & 31));
    d[0] = ph;
    d[16] = pl;
  }
  if (tid == 0) {
    float* tail = (float*)(wsp + (long long)Cout * K * 2);
    tail[co] = __int_as_float(-(er + ex));
    if (co == 0) tail[Cout] = ldexpf(1.f, ex);
  }
}

// *out = max |x| over the M x C f32 rows of pixel stride ldx (bit pattern of a non-negative float,
// so an integer max; *out zeroed by the caller)
// The f16 x3 pixel operand pre-split once per launch (conv_fwd_psplit_kernel SCH 8): out[p][cb] = the two
// f16 parts of x[p][32 cb .. 32 cb + 31] * s_x (split2h_8, exactly the kernel's own split), hi in bytes
// 0-63 and lo in 64-127 of the 128-B block; s_x is split_weight_h_kernel's (hsx, after the scales).  One
// thread per 8 channels.
__global__ __launch_bounds__(256) void split_x_h_kernel(const float* __restrict__ x, long long ldx, long long M,
                                                        int C, const float* __restrict__ hsx,
                                                        unsigned char* __restrict__ out) {
  const int c8 = C >> 3;
  const long long total = M * c8;
  const float s = *hsx;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long p = i / c8;
    const int q = (int)(i - p * c8);  // 8-channel group: block q >> 2, chunk q & 3
    const float* src = x + p * ldx + q * 8;
    const u4v x0 = *(const u4v*)src, x1 = *(const u4v*)(src + 4);
    s8v hi, lo;
    split2h_8(x0, x1, s, hi, lo);
    unsigned char* d = out + (p * (C >> 5) + (q >> 2)) * 128 + (q & 3) * 16;
    *(s8v*)d = hi;
    *(s8v*)(d + 64) = lo;
  }
}

__global__ __launch_bounds__(256) void amax_kernel(const float* __restrict__ x, long long ldx, long long M, int C,
                                                   unsigned* __restrict__ out) {
  __shared__ float red[4];
  const int cq = C >> 2;
  const long long total = M * cq;
  float m = 0.f;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long p = i / cq;
    const f4v v = *(const f4v*)(x + p * ldx + (i - p * cq) * 4);
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) amax_fold(out, fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

// Operand maxima with channels (dg_amax, and the f16 x3 weight gradients' per-channel scales where no
// producer supplied them): out[0] = max |x|, out[1 + c] = max over channel c (zeroed before).  A block
// takes G = min(C/4, 256) 16-byte channel chunks (blockIdx.y picks the group) x 256/G pixel rows, so
// each thread keeps its 4 channels in registers over a grid-stride pixel loop.
__global__ __launch_bounds__(256) void camax_kernel(const float* __restrict__ x, long long ldx, long long M, int C,
                                                    float* __restrict__ out) {
  const int cq = C >> 2;
  const int G = min(cq, 256), rows = 256 / G;
  const int tid = threadIdx.x, ch = blockIdx.y * G + tid % G, r = tid / G;
  const bool on = r < rows && ch < cq;
  float m[4] = {0.f, 0.f, 0.f, 0.f};
  if (on) {
    for (long long p = (long long)blockIdx.x * rows + r; p < M; p += (long long)gridDim.x * rows) {
      const f4v v = *(const f4v*)(x + p * ldx + ch * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) m[e] = fmaxf(m[e], fabsf(v[e]));
    }
  }
  block_camax_commit<4>(m, on ? ch * 4 : 0, C, out);
}

// Split-K finish: y = sum of the ksplit f32 partials (+ bias, + y if accumulate), stored
// as T, and — when part != NULL — the BN statistics partials of the stored values in the
// epilogue's format (one (n, mean, M2) row per 256-pixel block, two passes over registers).
// Block = 256 pixels x 64 channels, 1024 threads: one channel quad x 4 pixels (stride 64)
// each, so even the smallest layers put ~16 waves per tile in flight on the loads.
constexpr int SKR_PL = 64;
template <typename T>
__global__ __launch_bounds__(1024) void splitk_reduce_kernel(const float* __restrict__ kpart, int ksplit, int M,
                                                             int Cout, const float* __restrict__ bias,
                                                             T* __restrict__ y, long long ldy, int accumulate,
                                                             float* __restrict__ part, const float* escale,
                                                             const float* eshift, int eact) {
  constexpr int PXT = 256 / SKR_PL;
  __shared__ float sh[2][SKR_PL][64];
  const int tid = threadIdx.x, cq = tid & 15, pl = tid >> 4;
  const int px0 = blockIdx.x * 256, c0 = blockIdx.y * 64 + 4 * cq;
  const long long slab = (long long)M * Cout;
  float b[4] = {0.f, 0.f, 0.f, 0.f};
  if (bias) {
    const f4v bv = *(const f4v*)(bias + c0);
    b[0] = bv[0]; b[1] = bv[1]; b[2] = bv[2]; b[3] = bv[3];
  }
  float v[PXT][4];
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < PXT; ++k) {
    const int px = px0 + pl + SKR_PL * k;
    if (px >= M) {
      v[k][0] = v[k][1] = v[k][2] = v[k][3] = 0.f;
      continue;
    }
    const float* src = kpart + (long long)px * Cout + c0;
    f4v a = *(const f4v*)src;
    int sp = 1;
    for (; sp + 1 < ksplit; sp += 2) {  // two slabs in flight per step
      const f4v t0 = *(const f4v*)(src + sp * slab);
      const f4v t1 = *(const f4v*)(src + (sp + 1) * slab);
      a[0] += t0[0]; a[1] += t0[1]; a[2] += t0[2]; a[3] += t0[3];
      a[0] += t1[0]; a[1] += t1[1]; a[2] += t1[2]; a[3] += t1[3];
    }
    if (sp < ksplit) {
      const f4v t0 = *(const f4v*)(src + sp * slab);
      a[0] += t0[0]; a[1] += t0[1]; a[2] += t0[2]; a[3] += t0[3];
    }
    float o[4] = {a[0] + b[0], a[1] + b[1], a[2] + b[2], a[3] + b[3]};
    T* dst = y + (long long)px * ldy + c0;
    if (accumulate) {
      float q[4];
      ld4(dst, q);
      o[0] += q[0]; o[1] += q[1]; o[2] += q[2]; o[3] += q[3];
    }
    if (escale) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = fmaf(o[r], escale[c0 + r], eshift[c0 + r]);
        o[r] = (eact == 1 && !(t > 0.f)) ? 0.f : t;
      }
    }
    st4(dst, o);
    ++cnt;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[k][r] = Is16<T>::value ? round_to<T>(o[r]) : o[r];  // the stored value
      s[r] += v[k][r];
    }
  }
  if (!part) return;
  const int n = min(256, M - px0);
#pragma unroll
  for (int r = 0; r < 4; ++r) sh[0][pl][4 * cq + r] = s[r];
  __syncthreads();
  float mean[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float t = 0.f;
    for (int l = 0; l < SKR_PL; ++l) t += sh[0][l][4 * cq + r];
    mean[r] = t / (float)n;
  }
  float q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < PXT; ++k)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float d = v[k][r] - mean[r];
      q[r] = (k < cnt) ? fmaf(d, d, q[r]) : q[r];
    }
#pragma unroll
  for (int r = 0; r < 4; ++r) sh[1][pl][4 * cq + r] = q[r];
  __syncthreads();
  if (pl == 0) {
    float* row = part + (long long)blockIdx.x * 3 * Cout;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float m2 = 0.f;
      for (int l = 0; l < SKR_PL; ++l) m2 += sh[1][l][4 * cq + r];
      row[c0 + r] = (float)n;
      row[Cout + c0 + r] = mean[r];
      row[2 * Cout + c0 + r] = m2;
    }
  }
}

// K-slices for a pipelined bf16 forward whose tile grid cannot fill the chip (deep
// layers at small batch: 3k-25k pixels): the split minimising a cost model of the K loop
// against the reduce traffic, keeping one wave of blocks (<= 256, one 128-KB-LDS block per
// CU) and at least 3 K-steps per slice.
static int fwd_ksplit(long long M, int Cout, int C, int R, int S) {
  const char* e = getenv("DGVCC_SPLITK");
  if (e && e[0] == '0') return 1;
  if (C % 64 != 0) return 1;
  const int BN = Cout % 256 == 0 ? 256 : (Cout % 128 == 0 ? 128 : 64);
  if (Cout == 64 || BN == 64) return 1;
  const long long nblk = (M + 255) / 256 * (Cout / BN);
  if (nblk >= 128) return 1;
  const int KT = R * S * (C / 64);
  // cost model (us), measured on MI355X: ~2.2 us per K-step of a 256x256 tile (1.2 for
  // 128-wide), one wave of blocks; the reduce moves 8 B per partial element at ~4 TB/s.
  const double tstep = BN == 256 ? 2.2 : 1.2;
  const double red = (double)M * Cout * 8.0 / 4.0e6;
  int best = 1;
  double tbest = KT * tstep;
  const int smax = (int)std::min<long long>(256 / nblk, KT / 3);
  for (int ks = 2; ks <= std::min(smax, 32); ++ks) {
    const double t = (double)((KT + ks - 1) / ks) * tstep + 3.0 + ks * red;
    if (t < tbest) { tbest = t; best = ks; }
  }
  return best;
}

static int g_persist_override = -1;  // dg_set_persist (tests): -1 = environment / default
static bool use_persist() {
  if (g_persist_override >= 0) return g_persist_override == 1;
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DGVCC_PERSIST");
    v = (e && e[0] == '0') ? 0 : 1;  // default on: +1.0% on the 768x1024 step (A/B in one call)
  }
  return v == 1;
}

// DGVCC_SHORTK_REG=1: 16-bit forwards with <= 2 K-steps (the ResNet trunks' 1x1 convs from 64
// or 128 channels, HBM-bound) on the register-staged two-blocks-per-CU kernel (A/B switch)
static bool short_k_reg() {
  const char* e = getenv("DGVCC_SHORTK_REG");
  return e && e[0] == '1';
}

// DGVCC_F32_PERSIST=0: f32 forwards on the register-staged conv_fwd_kernel (A/B switch)
static bool use_f32_persist() {
  const char* e = getenv("DGVCC_F32_PERSIST");
  return !(e && e[0] == '0');
}
static int f32_pers_bn(int Cout);
static bool f32_pers_ok(const FwdArgs& a);
static bool f32_pers_shape_ok(const FwdArgs& a, int kmin);

// f32 GEMM arithmetic: 0 = v_mfma_f32_16x16x4_f32, 1 = the exact 3-way bf16 split on
// v_mfma_f32_16x16x32_bf16 (dg_common.h split3_8; f32-grade).
// Default: DGVCC_F32_MATH (exact | split | h16), else h16; dg_set_f32_math overrides.
// 2 (h16, default since round 5): the split math, with the f16 x3 arithmetic where a kernel has it
// (dg_common.h: the pre-split forward/dgrad, the 3-tap Cout = 64 forward, the split wgrads)
static int g_f32_math = -1;
static int f32_math() {
  if (g_f32_math < 0) {
    const char* e = getenv("DGVCC_F32_MATH");
    g_f32_math = (e && e[0] == 'e') ? 0 : (e && e[0] == 's') ? 1 : 2;
  }
  return g_f32_math;
}
static bool f32_split() { return f32_math() >= 1; }
static bool f32_h16() { return f32_math() == 2; }

static int persist_grid() {  // one block per CU (the ring takes most of the LDS)
  static int g = -1;
  if (g < 0) {
    const char* e = getenv("DGVCC_PERSIST_GRID");
    g = e ? std::max(8, atoi(e)) : 256;
  }
  return g;
}

static int pipe_var() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DGVCC_PIPE_VAR");
    v = e ? atoi(e) : 2;
  }
  return v;
}

static bool pipe_wide() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DGVCC_CONV_WIDE");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

static bool use_tap3() {
  const char* e = getenv("DGVCC_TAP3");
  return !(e && e[0] == '0');
}

static bool use_wgrad_pipe() {
  const char* e = getenv("DGVCC_WGRAD_PIPE");
  return e && e[0] == '1';
}

static bool use_pipe() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DGVCC_CONV_PIPE");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

// ---------------------------------------------------------------------------
// bf16 forward/dgrad for Cout = 64, 3x3 / stride 1 / pad 1, W % 256 == 0:
// a tile is 256 output pixels of ONE image row x 64 channels; a K-step is one
// kernel row dh and 64 input channels, staging the 3 taps' filters and ONE
// 264-pixel X strip that the 3 taps read at row offsets 0/1/2 (3x fewer staged
// X bytes than one tap per step).  Single LDS stage (57 KB), two blocks per CU
// overlap each other's loads and MFMAs.
// ---------------------------------------------------------------------------
constexpr int T3_XROWS = 264;

// Epilogue of the 3-tap kernels: bias / accumulate / eval-BN affine, bf16 store, and the
// per-256-pixel BN statistics row of the stored values.
template <int PADK, int TI, int TJ, int BN, int BM, typename Unpad, typename T = bf16>
__device__ __forceinline__ void tap3_epilogue(f4v (&acc)[TI][TJ], const FwdArgs& a, int px0, int wpx, int fr, int fc,
                                              int wid, int tid, char* smem, Unpad unpad) {
  T* y = (T*)a.y;
  bool valid[TJ];
  // bias read once, ahead of the stores (see conv_fwd_pipe_kernel); on the padded index the
  // extra 16 VGPRs spill the narrow kernel, so it keeps the per-use load there
  f4v bv[TI];
#pragma unroll
  for (int i = 0; i < TI; ++i)
    bv[i] = (!PADK && a.bias) ? *(const f4v*)(a.bias + 16 * i + 4 * fc) : f4v{0.f, 0.f, 0.f, 0.f};
  // accumulate, the eval-BN affine and (PADK) the per-use bias load run in a pass of their own
  // ahead of the stores, so the store loop holds no global loads (EPI_ACC_NOTE)
  const bool pre = a.accumulate || a.escale || (PADK && a.bias);
  if (pre) {
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int px = PADK ? unpad(px0 + wpx + 16 * j + fr) : px0 + wpx + 16 * j + fr;
      if (px < 0) continue;
      const T* yrow = y + (long long)px * a.ldy;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int co = 16 * i + 4 * fc;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if (a.bias) {
          const f4v b = PADK ? *(const f4v*)(a.bias + co) : bv[i];
          v[0] += b[0]; v[1] += b[1]; v[2] += b[2]; v[3] += b[3];
        }
        if (a.accumulate) add_old_y(v, yrow, a, px, co);
        epi_affine(v, a, co);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = v[r];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int px = PADK ? unpad(px0 + wpx + 16 * j + fr) : px0 + wpx + 16 * j + fr;
    valid[j] = px >= 0;  // unpadded path: M % 256 == 0
    if (px < 0) continue;
    T* yrow = y + (long long)px * a.ldy;
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int co = 16 * i + 4 * fc;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (!PADK && a.bias && !pre) {
        const f4v b = bv[i];
        v[0] += b[0]; v[1] += b[1]; v[2] += b[2]; v[3] += b[3];
      }
      st4(yrow + co, v);
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = round_to<T>(v[r]);  // the stored value, for the statistics
    }
  }
  if (a.part)
    epi_stats<TI, TJ, 4, BN>(acc, valid, wid, 0, smem, a.part + (long long)(px0 / BM) * 3 * a.Cout, a.Cout, 0, tid,
                             fr, fc);
}

// PADK = 1 (W % 256 != 0: 320-px crops, evaluation frames): the 256-wide tile runs over the
// zero-padded pixel index u = (n, p+1, q+1) in N x (H+2) x (W+2) instead of one image row, so
// a tile may span rows and images; each kernel row's X strip is contiguous in u and the taps'
// +-1 shifts land on zero pad cells exactly where the convolution pads.  Outputs on pad cells
// are computed and dropped ((H+2)(W+2)/HW more MFMA work: +1.3% at 320x320).
template <int PADK = 0, typename T = bf16>
__global__ __launch_bounds__(256, 2) void conv_fwd_tap3_kernel(FwdArgs a) {
  constexpr int BN = 64, BM = 256;
  constexpr int A_BYTES = 3 * BN * 128, X_BYTES = T3_XROWS * 128;
  constexpr int A_INST = A_BYTES / 1024, X_INST = X_BYTES / 1024;   // 24 + 33
  constexpr int N_INST = A_INST + X_INST;
  constexpr int TI = 4, TJ = 4;                                      // wave tile 64 px x 64 co
  __shared__ __attribute__((aligned(1024))) char smem[A_BYTES + X_BYTES];

  const int HW = a.H * a.W;
  const int M = a.N * HW;
  const int PW = a.W + 2, PHW = (a.H + 2) * PW;
  const int U = PADK ? a.N * PHW : M;
  const int px0 = xcd_remap(blockIdx.x, gridDim.x) * BM;  // tile origin (padded index when PADK)
  const int n = px0 / HW, rem = px0 - n * HW;
  const int pr = rem / a.W, q0 = rem - pr * a.W;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lrow = lane >> 3;
  const int xlo = PADK ? 0 : max(0, px0 - a.W - 8), xhi = PADK ? M : min(M, px0 + BM + a.W + 8);
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.x + (long long)xlo * a.ldx * 2), 0, (unsigned)(((long long)(xhi - xlo - 1) * a.ldx + a.C) * 2),
      0x00020000);
  auto unpad = [&](int u) -> int {  // padded index -> pixel, -1 on a pad cell / outside [0, U)
    if (u < 0 || u >= U) return -1;
    const int nn = u / PHW, r = u - nn * PHW;
    const int pp = r / PW, qq = r - pp * PW;
    if (pp < 1 || pp > a.H || qq < 1 || qq > a.W) return -1;
    return nn * HW + (pp - 1) * a.W + (qq - 1);
  };
  const long long ldw = 9ll * a.C;
  __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, (unsigned)(BN * ldw * 2), 0x00020000);
  const int CB = a.C / 64;
  const int KT = 3 * CB;

  f4v acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  const int wpx = wid * 64;
  const int fr = lane & 15, fc = lane >> 4;
  const char* As = smem;
  const char* Xs = smem + A_BYTES;

  for (int t = 0; t < KT; ++t) {
    const int dh = t % 3, cb = t / 3;
    for (int ii = wid; ii < N_INST; ii += 4) {
      if (ii < A_INST) {  // filter rows: tap s = ii / 8, co rows (ii % 8) * 8 + lrow
        const int sw = ii >> 3, row = (ii & 7) * 8 + lrow;
        const int ch = (lane & 7) ^ (row & 7);
        lds_dma16(wr, As + ii * 1024,
                  (unsigned)(((long long)row * ldw + (dh * 3 + sw) * a.C + cb * 64 + ch * 8) * 2));
      } else if (PADK) {  // X strip rows: padded index px0 - 4 + row of kernel row dh
        const int jj = ii - A_INST, row = jj * 8 + lrow;
        const int ch = (lane & 7) ^ (row & 7);
        const int pin = unpad(px0 - 4 + row + (dh - 1) * PW);
        lds_dma16(xr, Xs + jj * 1024,
                  pin >= 0 ? (unsigned)(((long long)pin * a.ldx + cb * 64 + ch * 8) * 2) : 0xFFFFFFF0u);
      } else {            // X strip rows: pixel q0 - 4 + row of image row pr + dh - 1
        const int jj = ii - A_INST, row = jj * 8 + lrow;
        const int ch = (lane & 7) ^ (row & 7);
        const int h = pr + dh - 1, w = q0 - 4 + row;
        const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
        const long long pin = (long long)n * HW + (long long)h * a.W + w - xlo;
        lds_dma16(xr, Xs + jj * 1024, ok ? (unsigned)((pin * a.ldx + cb * 64 + ch * 8) * 2) : 0xFFFFFFF0u);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int sw = 0; sw < 3; ++sw) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int ch = 4 * ks + fc;
        u4v af[TI], bfr[TJ];
#pragma unroll
        for (int j = 0; j < TJ; ++j) bfr[j] = *(const u4v*)(Xs + swz(wpx + 16 * j + fr + sw + 3, ch));
#pragma unroll
        for (int i = 0; i < TI; ++i) af[i] = *(const u4v*)(As + sw * BN * 128 + swz(16 * i + fr, ch));
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j) mfma_frag<T>(acc[i][j], af[i], bfr[j]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  tap3_epilogue<PADK, TI, TJ, BN, BM, decltype(unpad), T>(acc, a, px0, wpx, fr, fc, wid, tid, smem, unpad);
}

// Narrow-K 3-tap forward/dgrad (same tiles and outputs as conv_fwd_tap3_kernel): a K-step is
// one kernel row and 32 input channels, so LDS rows are 64 B and a block's single stage is
// 29 KB (filters 12 KB + a 272-pixel X strip 17 KB).  Five blocks per CU then keep five
// stages in flight where the 57 KB stage allowed two (the 64-wide kernel runs at ~28% MFMA
// busy, latency-bound).  Measured gain is small (~8% on these launches): the layer stages
// 110 FLOP per byte, so the bytes a CU must keep in flight exceed what its LDS can hold.  64-B rows are swizzled as chunk ^ 2*((row >> 2) & 1): for any row offset
// the 16 lanes of each ds_read_b128 group hit 16 distinct (row & 3, chunk) bank groups.
constexpr int T3N_XROWS = 272;
__device__ __forceinline__ int swz64(int row, int chunk) { return row * 64 + ((chunk ^ (((row >> 2) & 1) << 1)) << 4); }

template <int PADK = 0, typename T = bf16>
__global__ __launch_bounds__(256, 5) void conv_fwd_tap3n_kernel(FwdArgs a) {
  constexpr int BN = 64, BM = 256, BKC = 32;
  constexpr int A_BYTES = 3 * BN * 64, X_BYTES = T3N_XROWS * 64;
  constexpr int A_INST = A_BYTES / 1024, X_INST = X_BYTES / 1024;   // 12 + 17
  constexpr int N_INST = A_INST + X_INST;
  constexpr int TI = 4, TJ = 4;                                      // wave tile 64 px x 64 co
  __shared__ __attribute__((aligned(1024))) char smem[A_BYTES + X_BYTES];

  const int HW = a.H * a.W;
  const int M = a.N * HW;
  const int PW = a.W + 2, PHW = (a.H + 2) * PW;
  const int U = PADK ? a.N * PHW : M;
  const int px0 = xcd_remap(blockIdx.x, gridDim.x) * BM;
  const int n = px0 / HW, rem = px0 - n * HW;
  const int pr = rem / a.W, q0 = rem - pr * a.W;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lrow = lane >> 2;
  const int xlo = PADK ? 0 : max(0, px0 - a.W - 8), xhi = PADK ? M : min(M, px0 + BM + a.W + 8);
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.x + (long long)xlo * a.ldx * 2), 0, (unsigned)(((long long)(xhi - xlo - 1) * a.ldx + a.C) * 2),
      0x00020000);
  auto unpad = [&](int u) -> int {
    if (u < 0 || u >= U) return -1;
    const int nn = u / PHW, r = u - nn * PHW;
    const int pp = r / PW, qq = r - pp * PW;
    if (pp < 1 || pp > a.H || qq < 1 || qq > a.W) return -1;
    return nn * HW + (pp - 1) * a.W + (qq - 1);
  };
  const long long ldw = 9ll * a.C;
  __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, (unsigned)(BN * ldw * 2), 0x00020000);
  const int KT = 3 * (a.C / BKC);

  f4v acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  const int wpx = wid * 64;
  const int fr = lane & 15, fc = lane >> 4;
  const char* As = smem;
  const char* Xs = smem + A_BYTES;

  for (int t = 0; t < KT; ++t) {
    const int dh = t % 3, cb = t / 3;
    for (int ii = wid; ii < N_INST; ii += 4) {
      if (ii < A_INST) {  // filter rows: tap s = ii / 4, co rows (ii % 4) * 16 + lrow
        const int sw = ii >> 2, row = (ii & 3) * 16 + lrow;
        const int ch = (lane & 3) ^ (((row >> 2) & 1) << 1);
        lds_dma16(wr, smem + ii * 1024,
                  (unsigned)(((long long)row * ldw + (dh * 3 + sw) * a.C + cb * BKC + ch * 8) * 2));
      } else {
        const int jj = ii - A_INST, row = jj * 16 + lrow;
        const int ch = (lane & 3) ^ (((row >> 2) & 1) << 1);
        if (PADK) {
          const int pin = unpad(px0 - 4 + row + (dh - 1) * PW);
          lds_dma16(xr, smem + A_BYTES + jj * 1024,
                    pin >= 0 ? (unsigned)(((long long)pin * a.ldx + cb * BKC + ch * 8) * 2) : 0xFFFFFFF0u);
        } else {
          const int h = pr + dh - 1, w = q0 - 4 + row;
          const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
          const long long pin = (long long)n * HW + (long long)h * a.W + w - xlo;
          lds_dma16(xr, smem + A_BYTES + jj * 1024,
                    ok ? (unsigned)((pin * a.ldx + cb * BKC + ch * 8) * 2) : 0xFFFFFFF0u);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int sw = 0; sw < 3; ++sw) {
      u4v af[TI], bfr[TJ];
#pragma unroll
      for (int j = 0; j < TJ; ++j) bfr[j] = *(const u4v*)(Xs + swz64(wpx + 16 * j + fr + sw + 3, fc));
#pragma unroll
      for (int i = 0; i < TI; ++i) af[i] = *(const u4v*)(As + sw * BN * 64 + swz64(16 * i + fr, fc));
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) mfma_frag<T>(acc[i][j], af[i], bfr[j]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  tap3_epilogue<PADK, TI, TJ, BN, BM, decltype(unpad), T>(acc, a, px0, wpx, fr, fc, wid, tid, smem, unpad);
}

// Persistent 3-tap forward/dgrad for C = Cout = 64 on row-aligned tiles (the full-resolution
// layer enc1.3 and its dgrad, models/models.py:35-38).  conv_fwd_tap3_kernel stages 57 KB per
// K-step with one stage per block and waits on it (rocprofv3: waves wait 40% of their time,
// 28% MFMA-busy).  Here the whole 72-KB filter bank (3 kernel rows x 3 taps x 64 co) is
// staged once per block and stays resident, and a K-step streams only its 33-KB X strip
// through a two-slot ring that runs across tile boundaries: the next strip (possibly the next
// tile's first) is in flight during the current step's MFMAs and the epilogue's stores.
// One block of 8 waves per CU (2 per SIMD), wave tile 64 px x 32 co.  Per tile the K order
// (dh, tap, k-half) and the statistics merge are those of (conv_fwd_tap3_kernel<0, T>), so
// outputs and BN partials are bit-identical to it.  (A four-slot ring of 32-channel
// half-strips, three steps ahead, measured slower: 1.41 vs 1.35 ms on 16x768x1024: twice the
// barriers per tile cost more than the deeper lookahead gained.)
constexpr int T3P_FILT = 9 * 64 * 128;    // resident filters, 72 KB
constexpr int T3P_XS = T3_XROWS * 128;    // one X strip, 33 KB
template <int ROWS, typename T = bf16>
__global__ __launch_bounds__(512, 1) void conv_fwd_tap3p_kernel(FwdArgs a) {
  constexpr int BN = 64, BM = 256, TI = 2, TJ = 4;
  constexpr int X_INST = T3P_XS / 1024;   // 33 DMA instructions per strip
  constexpr int EPI_B = 4 * 3 * BN * 4;   // epi_stats scratch [4][3][BN] f32
  __shared__ __attribute__((aligned(1024))) char smem[T3P_FILT + 2 * T3P_XS + EPI_B + 3 * BN * 4];
  char* Ws = smem;
  char* Xring = smem + T3P_FILT;
  char* epi_lds = Xring + 2 * T3P_XS;
  // bias / eval-BN scale / shift staged in LDS once: a global load in the epilogue would make
  // the compiler drain vmcnt to 0 per use, i.e. wait for the in-flight strip DMA and every
  // earlier store of the tile (vector-memory operations retire in issue order)
  float* ebuf = (float*)(epi_lds + EPI_B);

  const int HW = a.H * a.W;
  const int M = a.N * HW;
  const int TPR = a.W / BM;                // W % 256 == 0 (and H % ROWS == 0)
  const int ntile = M / (BM * ROWS);
  const int G = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lrow = lane >> 3;
  int lin = blockIdx.x;
  if (lin >= ntile) return;
  if (tid < BN) {
    ebuf[tid] = a.bias ? a.bias[tid] : 0.f;
    ebuf[BN + tid] = a.escale ? a.escale[tid] : 1.f;
    ebuf[2 * BN + tid] = a.escale ? a.eshift[tid] : 0.f;
  }

  // resident filters: tap k = dh * 3 + sw at Ws + k * 8 KB, co rows swizzled as swz(row, chunk)
  {
    const long long ldw = 9ll * 64;
    __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)a.w, 0, (unsigned)(BN * ldw * 2), 0x00020000);
    for (int ii = wid; ii < 72; ii += 8) {
      const int k = ii >> 3, row = (ii & 7) * 8 + lrow;
      const int ch = (lane & 7) ^ (row & 7);
      lds_dma16(wr, Ws + ii * 1024, (unsigned)((row * ldw + k * 64 + ch * 8) * 2));
    }
  }

  struct Ctx {
    int px0, n, pr, q0, xlo;
    __amdgpu_buffer_rsrc_t xr;
  };
  auto setup = [&](int l, Ctx& c) {
    const int t = xcd_remap(l, ntile);
    const int rp = t / TPR;                  // row group: image rows pr .. pr + ROWS - 1
    c.q0 = (t - rp * TPR) * BM;
    c.n = rp / (a.H / ROWS);
    c.pr = (rp - c.n * (a.H / ROWS)) * ROWS;
    c.px0 = c.n * HW + c.pr * a.W + c.q0;
    c.xlo = max(0, c.px0 - a.W - 8);
    const int xhi = min(M, c.px0 + (ROWS - 1) * a.W + BM + a.W + 8);
    c.xr = __builtin_amdgcn_make_buffer_rsrc((void*)(a.x + (long long)c.xlo * a.ldx * 2), 0,
                                             (unsigned)(((long long)(xhi - c.xlo - 1) * a.ldx + a.C) * 2), 0x00020000);
  };
  // X strip s: pixels q0 - 4 + row (row < 264) of image row pr + s - 1 (kernel row s of
  // output row pr, kernel row s - 1 of output row pr + 1)
  auto issue = [&](const Ctx& c, int dh, int slot) {
    char* Xs = Xring + slot * T3P_XS;
    const int h = c.pr + dh - 1;
    for (int jj = wid; jj < X_INST; jj += 8) {
      const int row = jj * 8 + lrow;
      const int ch = (lane & 7) ^ (row & 7);
      const int w = c.q0 - 4 + row;
      const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      const long long pin = (long long)c.n * HW + (long long)h * a.W + w - c.xlo;
      lds_dma16(c.xr, Xs + jj * 1024, ok ? (unsigned)((pin * a.ldx + ch * 8) * 2) : 0xFFFFFFF0u);
    }
  };

  Ctx cur, nxt;
  setup(lin, cur);
  bool has_next = lin + G < ntile;
  if (has_next) setup(lin + G, nxt);
  const int wpx = (wid & 3) * 64, wco = (wid >> 2) * 32;
  const int fr = lane & 15, fc = lane >> 4;
  int gs = 0;  // K-steps consumed across all tiles of this block (ring slot = gs & 1)
  issue(cur, 0, 0);
  while (true) {
    constexpr int NS = ROWS + 2;  // strips per tile
    f4v acc[ROWS][TI][TJ];
#pragma unroll
    for (int r = 0; r < ROWS; ++r)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[r][i][j] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dh = 0; dh < NS; ++dh, ++gs) {
      // this step's strip (and, first time, the filters) have landed; every wave is done
      // reading the other slot (previous step)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (dh < NS - 1) issue(cur, dh + 1, (gs + 1) & 1);
      else if (has_next) issue(nxt, 0, (gs + 1) & 1);
      const char* Xs = Xring + (gs & 1) * T3P_XS;
#pragma unroll
      for (int sw = 0; sw < 3; ++sw) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int ch = 4 * ks + fc;
          u4v bfr[TJ];
#pragma unroll
          for (int j = 0; j < TJ; ++j) bfr[j] = *(const u4v*)(Xs + swz(wpx + 16 * j + fr + sw + 3, ch));
#pragma unroll
          for (int r = 0; r < ROWS; ++r) {  // output row pr + r takes this strip as kernel row dh - r
            const int kr = dh - r;
            if (kr < 0 || kr > 2) continue;
            const char* As = Ws + (kr * 3 + sw) * (BN * 128);
            u4v af[TI];
#pragma unroll
            for (int i = 0; i < TI; ++i) af[i] = *(const u4v*)(As + swz(wco + 16 * i + fr, ch));
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
              for (int j = 0; j < TJ; ++j) mfma_frag<T>(acc[r][i][j], af[i], bfr[j]);
            __builtin_amdgcn_s_setprio(0);
          }
        }
      }
    }
    // epilogue (the next strip's DMA is in flight)
    T* y = (T*)a.y;
    bool valid[TJ];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
    const int opx0 = cur.px0 + r * a.W;
    if (a.accumulate) {  // y += old y ahead of the stores (EPI_ACC_NOTE)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const T* yrow = y + (long long)(opx0 + wpx + 16 * j + fr) * a.ldy;
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int co = wco + 16 * i + 4 * fc;
          float o[4];
          ld4(yrow + co, o);
          if (a.bias) {
            const f4v b = *(const f4v*)(ebuf + co);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[r][i][j][e] += b[e];
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[r][i][j][e] += o[e];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      valid[j] = true;
      T* yrow = y + (long long)(opx0 + wpx + 16 * j + fr) * a.ldy;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int co = wco + 16 * i + 4 * fc;
        float v[4] = {acc[r][i][j][0], acc[r][i][j][1], acc[r][i][j][2], acc[r][i][j][3]};
        if (a.bias && !a.accumulate) {
          const f4v b = *(const f4v*)(ebuf + co);
          v[0] += b[0]; v[1] += b[1]; v[2] += b[2]; v[3] += b[3];
        }
        if (a.escale) {  // as epi_affine
          const f4v sc = *(const f4v*)(ebuf + BN + co), sf = *(const f4v*)(ebuf + 2 * BN + co);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float t = fmaf(v[e], sc[e], sf[e]);
            if (a.eact == 1) t = t > 0.f ? t : 0.f;
            v[e] = t;
          }
        }
        st4(yrow + co, v);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[r][i][j][e] = round_to<T>(v[e]);  // the stored value, for the statistics
      }
    }
    if (a.part)
      epi_stats<TI, TJ, 4, BN>(acc[r], valid, wid & 3, wco, epi_lds, a.part + (long long)(opx0 / BM) * 3 * a.Cout,
                               a.Cout, 0, tid, fr, fc);
    }
    if (!has_next) break;
    cur = nxt;
    lin += G;
    has_next = lin + G < ntile;
    if (has_next) setup(lin + G, nxt);
  }
}

// output rows per persistent 3-tap tile (DGVCC_TAP3P_ROWS=1|2|3; ROWS must divide H): ROWS output
// rows share ROWS + 2 strips, so each barrier-separated strip feeds more MFMAs (4 rows spill)
static int tap3p_rows() {
  const char* e = getenv("DGVCC_TAP3P_ROWS");
  return (e && e[0] == '1') ? 1 : (e && e[0] == '3') ? 3 : 2;
}

static bool use_tap3p() {
  const char* e = getenv("DGVCC_TAP3P");
  return !(e && e[0] == '0');
}

// K-step width of the 3-tap kernels: 64 channels on row-aligned tiles (768x1024: the 32-ch
// kernel's forwards were 0.27 ms/step faster but the step 0.07 ms slower, same-box A/B), 32 on
// the padded index (320-px final-mode training: +1%, conv 9.74 -> 9.51 ms/step).
// DGVCC_TAP3_BK=32|64 forces one.
static int tap3_bk(bool padk) {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DGVCC_TAP3_BK");
    v = e ? atoi(e) : 0;
  }
  return v == 32 || v == 64 ? v : (padk ? 32 : 64);
}

// the padded 3-tap variant: whole-tensor x descriptor (32-bit byte offsets), no split-K
static bool tap3_pad_ok(const FwdArgs& a) {
  const char* e = getenv("DGVCC_TAP3_PAD");
  if (e && e[0] == '0') return false;
  if (!use_tap3() || a.ksplit > 1 || a.W % 256 == 0 || a.bpart) return false;
  const long long M = (long long)a.N * a.H * a.W;
  return M * a.ldx * 2 < (1ll << 31) && (long long)a.N * (a.H + 2) * (a.W + 2) < (1ll << 30);
}

static int f32_pers_bn(int Cout) { return Cout % 256 == 0 && pipe_wide() ? 256 : (Cout % 128 == 0 ? 128 : 64); }

// DGVCC_PSPLIT=0: split-math f32 forwards split the filter per wave (conv_fwd_pers_kernel SPL=1)
static bool use_psplit() {
  const char* e = getenv("DGVCC_PSPLIT");
  return !(e && e[0] == '0');
}

static int psplit_tile_px(const FwdArgs& a);
// DGVCC_PSPLIT_MIN_TILES: fewest pre-split tiles a launch may have (default 128: half the CUs busy
// at split-math rates still beats the exact-f32 register-staged kernel, tools/ab_psplit_small.py);
// 0 = the persistent forward's own bound (more 256-pixel tiles than CUs)
static int psplit_min_tiles() {
  const char* e = getenv("DGVCC_PSPLIT_MIN_TILES");
  return e ? atoi(e) : 128;
}
// f32 split-math shapes served by conv_fwd_psplit_kernel (filter panel pre-split per launch)
// DGVCC_PSPLIT_SHORTK=0: not for launches of 2 K-steps per tile (the trunks' 1x1 convs from 64
// channels, which then take the exact-f32 register-staged kernel)
static bool psplit_shortk() {
  const char* e = getenv("DGVCC_PSPLIT_SHORTK");
  return !(e && e[0] == '0');
}
static bool psplit_ok(const FwdArgs& a) {
  if (!(use_psplit() && f32_split() && f32_pers_shape_ok(a, psplit_shortk() ? 2 : 3) && f32_pers_bn(a.Cout) >= 128 &&
        (long long)a.Cout * a.R * a.S * a.C * 6 < (1ll << 31)))
    return false;
  const int mt = psplit_min_tiles();
  if (mt <= 0) return f32_pers_ok(a);
  const long long M = (long long)a.N * a.H * a.W;
  return (long long)dg_cdiv(M, psplit_tile_px(a)) * (a.Cout / f32_pers_bn(a.Cout)) >= mt;
}

// The f16 x3 pre-split forward reads its pixel operand pre-split by split_x_h_kernel (SCH 8) when
// several output-channel tiles share each pixel tile of a 3x3 conv (Cout > the tile's bn): each of those
// blocks would split the same fragments again, and the pass (8 B per element of HBM traffic) pays for
// itself; with one channel tile, or a 1x1 conv's short K, the in-kernel split (SCH 0) is faster
// (profiles/round5e/ab_xs/shapes_*).  DGVCC_PSPLIT_XS=0: never, =2: every eligible launch (A/B); read
// per launch.
static bool psplit_xs(const FwdArgs& a, int bn) {
  const char* e = getenv("DGVCC_PSPLIT_XS");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '2') return true;
  return a.Cout > bn && a.R * a.S > 1;
}
// workspace bytes of the pre-split pixel operand (after the filter planes, 256-B aligned)
static long long xsplit_bytes(const FwdArgs& a) { return (long long)a.N * a.H * a.W * a.C * 4; }
static long long xsplit_off(long long planes) { return (planes + 255) / 256 * 256; }

// DGVCC_PSPLIT_TALL=0: never the 256-pixel pre-split tiles; 1 (default): where they quantise onto the
// CUs no worse than the 192-pixel ones; 2: always (256-channel training forwards/dgrads)
static int psplit_tall_mode() {
  const char* e = getenv("DGVCC_PSPLIT_TALL");
  return e ? e[0] - '0' : 1;
}
// the 256-pixel form for this launch: 256 output channels, no eval epilogue, and (mode 1) whole
// rounds of 256-pixel tiles costing no more than the 192-pixel ones at ~5% less time per pixel
static bool psplit_tall(const FwdArgs& a) {
  const int mode = psplit_tall_mode();
  if (mode == 0 || f32_pers_bn(a.Cout) != 256 || a.escale || a.bpart || !psplit_inc()) return false;
  if (mode == 2) return true;
  const long long M = (long long)a.N * a.H * a.W, nco = a.Cout / 256, G = persist_grid();
  const long long r256 = dg_cdiv(dg_cdiv(M, 256) * nco, G), r192 = dg_cdiv(dg_cdiv(M, PSB) * nco, G);
  return (double)r256 * 256 * 0.95 < (double)r192 * PSB;
}
// pixels per tile of the pre-split launch (and so rows of its epilogue statistics)
static int psplit_tile_px(const FwdArgs& a) { return psplit_tall(a) ? 256 : psplit_psb(f32_pers_bn(a.Cout), psplit_wide()); }

// f32 split-math shapes served by conv_fwd_rsplit_kernel (64-wide channel tiles)
static bool rsplit_ok(const FwdArgs& a) {
  return use_psplit() && f32_split() && a.ksplit <= 1 && !a.bpart && a.C % 32 == 0 && a.ldx % 4 == 0 &&
         a.Cout % 64 == 0 && f32_pers_bn(a.Cout) == 64 && (long long)a.Cout * a.R * a.S * a.C * 6 < (1ll << 31);
}

// rows of W % 256 == 0 of a 3x3 / pad-1 Cout = 64 conv: the 3-tap strip kernel (DGVCC_RSPLIT3=0 off;
// =1 only the 256-pixel 2 x 4-wave form; default 2: the 512-pixel all-pixel-wave form where W % 512 == 0)
static int rsplit3_mode() {
  const char* e = getenv("DGVCC_RSPLIT3");
  return e ? e[0] - '0' : 2;
}
static bool rsplit3_ok(const FwdArgs& a) {
  return rsplit3_mode() != 0 && a.R == 3 && a.S == 3 && a.pad == 1 && a.W % 256 == 0;
}
static bool rsplit3w_ok(const FwdArgs& a) { return rsplit3_ok(a) && rsplit3_mode() == 2 && a.W % 512 == 0; }

// The pre-split filter planes of a split-math f32 launch: split_weight_kernel writes them into
// the caller's workspace (dg_conv_fwd_workspace) ahead of the conv on the same stream; null
// when the caller passed no room for them (the launch then takes a kernel that splits per wave).
static const unsigned short* presplit(const FwdArgs& a, hipStream_t st) {
  const long long nw = (long long)a.Cout * a.R * a.S * a.C;
  if (!a.wsplit || a.wsplit_bytes < nw * 6) return nullptr;
  unsigned short* wsp = (unsigned short*)a.wsplit;
  hipLaunchKernelGGL(split_weight_kernel, dim3((unsigned)std::min<long long>(dg_cdiv(nw, 256), 4096)), dim3(256), 0,
                     st, (const float*)a.w, nw, wsp);
  return wsp;
}
// DGVCC_PSPLIT_SCH=0..9 (read per launch: A/B): schedule of the f16 x3 256-pixel pre-split forward
// (conv_fwd_psplit_kernel SCH) where the pixel operand is not pre-split by its own pass; default 9 (the
// split once per block in LDS: 256->256 at 192x256 2.444 -> 2.397 ms, 512->256 dgrad 4.945 -> 4.871,
// bit-identical; profiles/round6e/ab_sch.txt)
static int psplit_sch() {
  const char* e = getenv("DGVCC_PSPLIT_SCH");
  return e ? e[0] - '0' : 9;
}
// test hook: the diagnostic stamp buffer (dg_debug_stamps)
static unsigned long long* g_stamps = nullptr;
static long long g_stamp_bytes = 0;
static int launch_amax(const float* x, long long ldx, long long M, int C, unsigned* out, hipStream_t st) {
  if (hipMemsetAsync(out, 0, 4, st) != hipSuccess) return DG_ERR_HIP;
  if (M <= 0) return DG_OK;
  hipLaunchKernelGGL(amax_kernel, dim3((unsigned)std::min<long long>(dg_cdiv(M * (C / 4), 256), 2048)), dim3(256), 0,
                     st, x, ldx, M, C, out);
  DG_CHECK_LAUNCH();
  return DG_OK;
}
// out [1 + C]: the tensor's max and each channel's (camax_kernel), ~1024 blocks
static int launch_camax(const float* x, long long ldx, long long M, int C, unsigned* out, hipStream_t st) {
  if (C % 4 != 0 || C > DG_CAMAX_C) return DG_ERR_UNSUPPORTED;
  if (hipMemsetAsync(out, 0, dg_amax_words(C) * 4, st) != hipSuccess) return DG_ERR_HIP;
  if (M <= 0) return DG_OK;
  const int cq = C / 4, G = std::min(cq, 256), rows = 256 / G, gy = dg_cdiv(cq, G);
  const int gx = (int)std::max(1LL, std::min<long long>(dg_cdiv(M, rows), std::max(1, 1024 / gy)));
  hipLaunchKernelGGL(camax_kernel, dim3(gx, gy), dim3(256), 0, st, x, ldx, M, C, (float*)out);
  DG_CHECK_LAUNCH();
  return DG_OK;
}
// f16 x3 planes + scales (split_weight_h_kernel) in the same workspace (Cout * K * 4 bytes of
// planes + 2 * Cout + 2 floats of scales, then the pixel operand's amax word): the x amax pass,
// then the filter split
static long long presplit_h_bytes(const FwdArgs& a) {
  return (long long)a.Cout * a.R * a.S * a.C * 4 + (2LL * a.Cout + 4) * 4;
}
static const unsigned short* presplit_h(const FwdArgs& a, hipStream_t st) {
  const long long K = (long long)a.R * a.S * a.C;
  if (!a.wsplit || a.wsplit_bytes < presplit_h_bytes(a)) return nullptr;
  unsigned short* wsp = (unsigned short*)a.wsplit;
  const unsigned* xam = (const unsigned*)a.xamax;
  if (!xam) {
    unsigned* slot = (unsigned*)(a.wsplit + a.Cout * K * 4 + (2LL * a.Cout + 2) * 4);
    if (launch_amax((const float*)a.x, a.ldx, (long long)a.N * a.H * a.W, a.C, slot, st) != DG_OK) return nullptr;
    xam = slot;
  }
  hipLaunchKernelGGL(split_weight_h_kernel, dim3((unsigned)a.Cout), dim3(256), 0, st, (const float*)a.w, (int)K, wsp,
                     (const unsigned*)xam, a.Cout);
  return wsp;
}
static bool has_split_room(const FwdArgs& a) {
  return a.wsplit && a.wsplit_bytes >= (long long)a.Cout * a.R * a.S * a.C * 6;
}

// the shapes the f32 persistent forward serves (and so the f32 shapes with epilogue statistics):
// more tiles than CUs, > PF K-steps per tile, no split-K / BN-backward epilogue
// kmin: fewest 32-channel K-steps per tile (the exact / per-wave-split persistent forward prefetches
// two K-steps of a tile in its prologue and needs > 2; the pre-split one needs >= its stage count - 1)
static bool f32_pers_shape_ok(const FwdArgs& a, int kmin) {
  return use_f32_persist() && use_persist() && inc_shape_ok(a) && a.ksplit <= 1 && !a.bpart && a.C % 32 == 0 &&
         a.ldx % 4 == 0 && a.Cout % 64 == 0 && a.Cout <= PERS_BIAS_MAX && a.R * a.S * (a.C / 32) >= kmin &&
         (long long)a.Cout * a.R * a.S * a.C * 4 < (1ll << 31);
}
static bool f32_pers_ok(const FwdArgs& a) {
  if (!f32_pers_shape_ok(a, 3)) return false;
  const long long M = (long long)a.N * a.H * a.W;
  return (long long)dg_cdiv(M, PBM) * (a.Cout / f32_pers_bn(a.Cout)) > 256;
}

static int conv_korder() {  // DGVCC_CONV_KORDER=0/1 (read per launch: same-process A/B)
  const char* e = getenv("DGVCC_CONV_KORDER");
  return e ? (e[0] == '1' ? 1 : 0) : 1;  // default channel-block-major (tools/ab_korder.py: f32 +2.5%, bf16 +4.3%)
}

template <typename T>
int launch_fwd_impl(const FwdArgs& a, hipStream_t st);

static bool pers_wide_on() {  // DGVCC_PERS_WIDE=0: the 16-bit 128-channel persistent forward on 2 x 4 waves
  const char* e = getenv("DGVCC_PERS_WIDE");
  return !(e && e[0] == '0');
}
// the 16-bit forward takes conv_fwd_pers_kernel<128, .., WIDE = 1> (384-pixel tiles): the same
// conditions as launch_fwd_impl's persistent branch at BN = 128, no split-K / BN-backward epilogue
// DGVCC_PERS_SHORTK=0: the 16-bit persistent forward only for > 2 K-steps per tile (round 3); default:
// down to the pipeline depth (1 K-step on the 2-stage kernels, 2 on the 3-stage ones), so the
// trunks' 1x1 convs from 64 / 128 channels run persistent too (read per launch: A/B)
static bool pers16_shortk() {
  const char* e = getenv("DGVCC_PERS_SHORTK");
  return !(e && e[0] == '0');
}
static int pers16_kmin(int stg) { return pers16_shortk() ? stg - 1 : 3; }
// DGVCC_PERS_WIDE_SMALL=0: 256-channel launches of <= 2 rounds of tiles stay on the pipe kernel
// (read per launch: A/B)
static bool pers_wide_small() {
  const char* e = getenv("DGVCC_PERS_WIDE_SMALL");
  return !(e && e[0] == '0');
}
static bool pers16_wide(const FwdArgs& a) {
  if (!(pers_wide_on() && use_pipe() && a.C % 64 == 0 && a.ldx % 8 == 0 &&
        !(short_k_reg() && a.R * a.S * (a.C / 64) <= 2) && (long long)a.Cout * a.R * a.S * a.C * 2 < (1ll << 31) &&
        a.ksplit <= 1 && !a.bpart && use_persist() && pipe_var() == 2 && inc_shape_ok(a) &&
        a.R * a.S * (a.C / 64) >= pers16_kmin(2) && a.Cout <= PERS_BIAS_MAX))
    return false;
  if (a.Cout % 128 != 0) return false;
  const long long M = (long long)a.N * a.H * a.W;
  if (!(a.Cout % 256 == 0 && pipe_wide())) return (long long)dg_cdiv(M, PBM) * (a.Cout / 128) > 2 * 256;  // BN = 128
  // 256-channel launches too small for the 256-channel persistent forward (<= 2 rounds of 256 x 256
  // tiles, which then ran one tile per block on the pipe kernel: 384 tiles = 1.5 rounds at 1/16
  // resolution): the 384 x 128 tiles where they cost fewer tile-areas of rounds (+10% for the
  // narrower tile's lower rate)
  // (grids small enough for split-K keep it: dg_conv_fwd_ex splits their K loop when given a
  // workspace, and the statistics rows must not depend on whether one was given)
  if (!pers_wide_small() || fwd_ksplit(M, a.Cout, a.C, a.R, a.S) > 1) return false;
  const long long t256 = (long long)dg_cdiv(M, PBM) * (a.Cout / 256);
  if (t256 > 2 * 256) return false;
  const long long tw = (long long)dg_cdiv(M, 384) * (a.Cout / 128), G = persist_grid();
  return (double)dg_cdiv(tw, G) * 384 * 128 * 1.1 < (double)dg_cdiv(t256, G) * 256 * 256;
}

// DGVCC_PERS_WST=0: the 8-byte epilogue stores; 1: 16-byte stores on the 1-2-K-step launches only;
// 2: every 256-channel / 384 x 128 16-bit persistent launch (bf16 final step +1.9%, 1x1 64 -> 256
// convs 1.34x); default 3: the 128- / 64-channel 3-stage ones too (SW bf16 step -0.7%); read per
// launch: A/B
static int pers_wst() {
  const char* e = getenv("DGVCC_PERS_WST");
  return e ? e[0] - '0' : 3;
}
template <typename T>
int launch_fwd(const FwdArgs& a0, hipStream_t st) {
  FwdArgs a = a0;
  a.korder = conv_korder();
  // 16-byte epilogue stores: a template variant (WST = 1) of the persistent kernel, not a run-time
  // branch -- both store forms in one instantiation pushed the 256-channel kernel past 256 VGPRs
  // (bit 0: the persistent kernels' WST instantiations; bit 1: the pipe kernel's run-time branch,
  // opt-in with DGVCC_PIPE_WST=1: bit-identical (test_pipe_wide_stores) but no faster on the bf16 final
  // step or the SW trunk, same-box A/B in profiles/round5a/pipe_wst/)
  a.wide_st = Is16<T>::value && pers_wst() > 0 && a.ldy % 8 == 0 && ((uintptr_t)a.y & 15) == 0 &&
              (pers_wst() >= 2 || a.R * a.S * (a.C / 64) <= 2);
  if (a.wide_st && getenv("DGVCC_PIPE_WST") && getenv("DGVCC_PIPE_WST")[0] == '1') a.wide_st |= 2;
  return launch_fwd_impl<T>(a, st);
}

template <typename T>
int launch_fwd_impl(const FwdArgs& a, hipStream_t st) {
  const long long M = (long long)a.N * a.H * a.W;
  if constexpr (Is16<T>::value) {
    if (use_pipe() && a.C % 64 == 0 && a.ldx % 8 == 0 && !(short_k_reg() && a.R * a.S * (a.C / 64) <= 2) &&
        (long long)a.Cout * a.R * a.S * a.C * 2 < (1ll << 31)) {
      const int np = dg_cdiv(M, PBM);
      const int var = pipe_var();
      const int epi = a.ksplit > 1 ? 1 : a.bpart ? 2 : a.escale ? 3 : 0;
#define PIPE_LAUNCH(BN_, STG_, G_) \
      do { \
        if (epi == 1) hipLaunchKernelGGL((conv_fwd_pipe_kernel<BN_, STG_, 2, 1, T>), dim3(G_), dim3(512), 0, st, a); \
        else if (epi == 2) hipLaunchKernelGGL((conv_fwd_pipe_kernel<BN_, STG_, 2, 2, T>), dim3(G_), dim3(512), 0, st, a); \
        else if (epi == 3) hipLaunchKernelGGL((conv_fwd_pipe_kernel<BN_, STG_, 2, 3, T>), dim3(G_), dim3(512), 0, st, a); \
        else if (var == 1) hipLaunchKernelGGL((conv_fwd_pipe_kernel<BN_, STG_, 1, 0, T>), dim3(G_), dim3(512), 0, st, a); \
        else if (var == 2) hipLaunchKernelGGL((conv_fwd_pipe_kernel<BN_, STG_, 2, 0, T>), dim3(G_), dim3(512), 0, st, a); \
        else hipLaunchKernelGGL((conv_fwd_pipe_kernel<BN_, STG_, 0, 0, T>), dim3(G_), dim3(512), 0, st, a); \
      } while (0)
      if (a.ksplit > 1) {  // BN and stage count as the unsplit choice below
        const unsigned g = (unsigned)(np * (a.Cout / (a.Cout % 256 == 0 && pipe_wide() ? 256 : 128)) * a.ksplit);
        if (a.Cout % 256 == 0 && pipe_wide()) PIPE_LAUNCH(256, 2, g);
        else PIPE_LAUNCH(128, 3, g);
        DG_CHECK_LAUNCH();
        hipLaunchKernelGGL(splitk_reduce_kernel<T>, dim3((unsigned)dg_cdiv(M, 256), a.Cout / 64), dim3(1024), 0, st,
                           (const float*)a.kpart, a.ksplit, (int)M, a.Cout, a.bias, (T*)a.y, a.ldy, a.accumulate,
                           a.part, a.escale, a.eshift, a.eact);
      } else if (a.Cout == 64 && a.R == 3 && a.S == 3 && a.pad == 1 && a.W % 256 == 0 && use_tap3()) {
        if (a.C == 64 && !a.bpart && use_tap3p()) {
          const unsigned g = (unsigned)std::min<long long>(M / 256, persist_grid());
          if (a.H % 3 == 0 && tap3p_rows() == 3)
            hipLaunchKernelGGL((conv_fwd_tap3p_kernel<3, T>), dim3((unsigned)std::min<long long>(M / 768, g)), dim3(512), 0, st, a);
          else if (a.H % 2 == 0 && tap3p_rows() >= 2)
            hipLaunchKernelGGL((conv_fwd_tap3p_kernel<2, T>), dim3((unsigned)std::min<long long>(M / 512, g)), dim3(512), 0, st, a);
          else
            hipLaunchKernelGGL((conv_fwd_tap3p_kernel<1, T>), dim3(g), dim3(512), 0, st, a);
        } else if (tap3_bk(false) == 32) hipLaunchKernelGGL((conv_fwd_tap3n_kernel<0, T>), dim3((unsigned)(M / 256)), dim3(256), 0, st, a);
        else hipLaunchKernelGGL((conv_fwd_tap3_kernel<0, T>), dim3((unsigned)(M / 256)), dim3(256), 0, st, a);
      } else if (a.Cout == 64 && a.R == 3 && a.S == 3 && a.pad == 1 && !a.part && tap3_pad_ok(a)) {
        const long long U = (long long)a.N * (a.H + 2) * (a.W + 2);
        if (tap3_bk(true) == 32) hipLaunchKernelGGL((conv_fwd_tap3n_kernel<1, T>), dim3((unsigned)dg_cdiv(U, 256)), dim3(256), 0, st, a);
        else hipLaunchKernelGGL((conv_fwd_tap3_kernel<1, T>), dim3((unsigned)dg_cdiv(U, 256)), dim3(256), 0, st, a);
      } else if (use_persist() && !a.bpart && var == 2 && inc_shape_ok(a) &&
                 a.R * a.S * (a.C / 64) >= pers16_kmin(a.Cout % 256 == 0 && pipe_wide() ? 2 : 3) && a.Cout <= PERS_BIAS_MAX &&
                 (long long)np * (a.Cout / (a.Cout % 256 == 0 && pipe_wide() ? 256 : (a.Cout % 128 == 0 ? 128 : 64))) >
                     2 * 256) {
        const int bn = a.Cout % 256 == 0 && pipe_wide() ? 256 : (a.Cout % 128 == 0 ? 128 : 64);
        const long long tiles = (long long)np * (a.Cout / bn);
        const unsigned g = (unsigned)std::min<long long>(tiles, persist_grid());
        if (epi == 3) {
          if (bn == 256) hipLaunchKernelGGL((conv_fwd_pers_kernel<256, 2, 3, T>), dim3(g), dim3(512), 0, st, a);
          else if (bn == 128) hipLaunchKernelGGL((conv_fwd_pers_kernel<128, 3, 3, T>), dim3(g), dim3(512), 0, st, a);
          else hipLaunchKernelGGL((conv_fwd_pers_kernel<64, 3, 3, T>), dim3(g), dim3(512), 0, st, a);
        } else if (bn == 128 && pers16_wide(a)) {
          const unsigned gw = (unsigned)std::min<long long>((long long)dg_cdiv(M, 384) * (a.Cout / 128), persist_grid());
          if (a.wide_st) hipLaunchKernelGGL((conv_fwd_pers_kernel<128, 2, 0, T, 0, 1, 1, 1>), dim3(gw), dim3(512), 0, st, a);
          else hipLaunchKernelGGL((conv_fwd_pers_kernel<128, 2, 0, T, 0, 1, 1>), dim3(gw), dim3(512), 0, st, a);
        } else {
          if (!pers_inc()) {  // A/B: per-K-step recomputed DMA addressing
            if (bn == 256) hipLaunchKernelGGL((conv_fwd_pers_kernel<256, 2, 0, T, 0, 0>), dim3(g), dim3(512), 0, st, a);
            else if (bn == 128) hipLaunchKernelGGL((conv_fwd_pers_kernel<128, 3, 0, T, 0, 0>), dim3(g), dim3(512), 0, st, a);
            else hipLaunchKernelGGL((conv_fwd_pers_kernel<64, 3, 0, T, 0, 0>), dim3(g), dim3(512), 0, st, a);
          } else if (bn == 256 && a.wide_st) hipLaunchKernelGGL((conv_fwd_pers_kernel<256, 2, 0, T, 0, 1, 0, 1>), dim3(g), dim3(512), 0, st, a);
          else if (bn == 256) hipLaunchKernelGGL((conv_fwd_pers_kernel<256, 2, 0, T>), dim3(g), dim3(512), 0, st, a);
          else if (bn == 128 && a.wide_st && pers_wst() == 3)
            hipLaunchKernelGGL((conv_fwd_pers_kernel<128, 3, 0, T, 0, 1, 0, 1>), dim3(g), dim3(512), 0, st, a);
          else if (bn == 128) hipLaunchKernelGGL((conv_fwd_pers_kernel<128, 3, 0, T>), dim3(g), dim3(512), 0, st, a);
          else if (a.wide_st && pers_wst() == 3)
            hipLaunchKernelGGL((conv_fwd_pers_kernel<64, 3, 0, T, 0, 1, 0, 1>), dim3(g), dim3(512), 0, st, a);
          else hipLaunchKernelGGL((conv_fwd_pers_kernel<64, 3, 0, T>), dim3(g), dim3(512), 0, st, a);
        }
      } else if (epi == 0 && pers16_wide(a)) {  // small 256-channel grids on 384 x 128 persistent tiles
        const unsigned gw = (unsigned)std::min<long long>((long long)dg_cdiv(M, 384) * (a.Cout / 128), persist_grid());
        if (a.wide_st) hipLaunchKernelGGL((conv_fwd_pers_kernel<128, 2, 0, T, 0, 1, 1, 1>), dim3(gw), dim3(512), 0, st, a);
        else hipLaunchKernelGGL((conv_fwd_pers_kernel<128, 2, 0, T, 0, 1, 1>), dim3(gw), dim3(512), 0, st, a);
      } else if (a.Cout % 256 == 0 && pipe_wide()) PIPE_LAUNCH(256, 2, np * (a.Cout / 256));
      else if (a.Cout % 128 == 0) PIPE_LAUNCH(128, 3, np * (a.Cout / 128));
      else PIPE_LAUNCH(64, 3, np * (a.Cout / 64));
#undef PIPE_LAUNCH
      DG_CHECK_LAUNCH();
      return DG_OK;
    }
  }
  if constexpr (!Is16<T>::value) {
    if (a.bpart) {  // dgrad with the BN-backward partials in the epilogue: the pre-split kernel only
      FwdArgs q = a;
      q.bpart = nullptr;
      if (!(psplit_ok(q) && psplit_wide() && has_split_room(a))) return DG_ERR_UNSUPPORTED;
      const bool h16 = f32_h16();
      const unsigned short* wsp = h16 ? presplit_h(a, st) : presplit(a, st);
      if (!wsp) return DG_ERR_HIP;
      const int bn2 = f32_pers_bn(a.Cout);
      const unsigned g2 = (unsigned)std::min<long long>((long long)dg_cdiv(M, psplit_psb(bn2)) * (a.Cout / bn2),
                                                        persist_grid());
      if (h16) {
        if (bn2 == 256) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 2, 1, 1, 0, 1>), dim3(g2), dim3(512), 0, st, a, (const char*)wsp);
        else hipLaunchKernelGGL((conv_fwd_psplit_kernel<128, 2, 2, 1, 1, 0, 1>), dim3(g2), dim3(512), 0, st, a, (const char*)wsp);
      } else if (bn2 == 256) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 2>), dim3(g2), dim3(512), 0, st, a, (const char*)wsp);
      else hipLaunchKernelGGL((conv_fwd_psplit_kernel<128, 2, 2>), dim3(g2), dim3(512), 0, st, a, (const char*)wsp);
      DG_CHECK_LAUNCH();
      return DG_OK;
    }
    if (rsplit_ok(a) && has_split_room(a)) {  // split math, Cout = 64: both operands split once per block
      // f16 x3 on the 512-pixel 3-tap form; the 256-pixel 3-tap and per-tap forms (W % 512 != 0: the trunks'
      // and 320-px crops' Cout = 64 layers) stay on the bf16 x6 split unless DGVCC_RSPLIT_H16=1 (read per
      // launch): with f16 x3 there, models2 DensityRegressorM's forward_train density map at 2 x 64 x 64
      // moved from 6.5e-5 to 1.06e-4 of float64 (budget 1e-4; the fp32 torch reference's own 3.4e-5),
      // measured round 6
      const char* eh = getenv("DGVCC_RSPLIT_H16");
      const bool h16 = f32_h16() && (rsplit3w_ok(a) || (eh && eh[0] == '1'));
      const unsigned short* wsp = h16 ? presplit_h(a, st) : presplit(a, st);
      if (!wsp) return DG_ERR_HIP;
      const dim3 g((unsigned)((long long)dg_cdiv(M, 256) * (a.Cout / 64)));
      const char* ws = (const char*)wsp;
      if (rsplit3w_ok(a)) {
        const dim3 gw((unsigned)((long long)(M / 512) * (a.Cout / 64)));
        if (h16 && a.escale) hipLaunchKernelGGL((conv_fwd_rsplit3w_kernel<3, 1>), gw, dim3(512), 0, st, a, ws);
        else if (h16) hipLaunchKernelGGL((conv_fwd_rsplit3w_kernel<0, 1>), gw, dim3(512), 0, st, a, ws);
        else if (a.escale) hipLaunchKernelGGL((conv_fwd_rsplit3w_kernel<3>), gw, dim3(512), 0, st, a, ws);
        else hipLaunchKernelGGL((conv_fwd_rsplit3w_kernel<0>), gw, dim3(512), 0, st, a, ws);
      } else if (rsplit3_ok(a)) {
        if (h16 && a.escale) hipLaunchKernelGGL((conv_fwd_rsplit3_kernel<3, 1>), g, dim3(512), 0, st, a, ws);
        else if (h16) hipLaunchKernelGGL((conv_fwd_rsplit3_kernel<0, 1>), g, dim3(512), 0, st, a, ws);
        else if (a.escale) hipLaunchKernelGGL((conv_fwd_rsplit3_kernel<3>), g, dim3(512), 0, st, a, ws);
        else hipLaunchKernelGGL((conv_fwd_rsplit3_kernel<0>), g, dim3(512), 0, st, a, ws);
      } else if (h16 && a.escale) hipLaunchKernelGGL((conv_fwd_rsplit_kernel<3, 1>), g, dim3(512), 0, st, a, ws);
      else if (h16) hipLaunchKernelGGL((conv_fwd_rsplit_kernel<0, 1>), g, dim3(512), 0, st, a, ws);
      else if (a.escale) hipLaunchKernelGGL((conv_fwd_rsplit_kernel<3>), g, dim3(512), 0, st, a, ws);
      else hipLaunchKernelGGL((conv_fwd_rsplit_kernel<0>), g, dim3(512), 0, st, a, ws);
      DG_CHECK_LAUNCH();
      return DG_OK;
    }
    // f32: the persistent LDS-DMA pipeline with 128-B (32-channel) K-steps; each K-step is 4x
    // the MFMA work of a 16-bit one (v_mfma_f32_16x16x4_f32), so the 2-stage 256-wide ring
    // hides the DMA latency comfortably.  Epilogue BN statistics (a.part) as in 16-bit.
    if (f32_pers_ok(a) || (psplit_ok(a) && has_split_room(a))) {
      const int np = dg_cdiv(M, PBM);
      const int bn = f32_pers_bn(a.Cout);
      const long long tiles = (long long)np * (a.Cout / bn);
      const unsigned g = (unsigned)std::min<long long>(tiles, persist_grid());
#define F32_PERS(SPL_) \
      do { \
        if (a.escale) { \
          if (bn == 256) hipLaunchKernelGGL((conv_fwd_pers_kernel<256, 2, 3, T, SPL_>), dim3(g), dim3(512), 0, st, a); \
          else if (bn == 128) hipLaunchKernelGGL((conv_fwd_pers_kernel<128, 3, 3, T, SPL_>), dim3(g), dim3(512), 0, st, a); \
          else hipLaunchKernelGGL((conv_fwd_pers_kernel<64, 3, 3, T, SPL_>), dim3(g), dim3(512), 0, st, a); \
        } else { \
          if (bn == 256) hipLaunchKernelGGL((conv_fwd_pers_kernel<256, 2, 0, T, SPL_>), dim3(g), dim3(512), 0, st, a); \
          else if (bn == 128) hipLaunchKernelGGL((conv_fwd_pers_kernel<128, 3, 0, T, SPL_>), dim3(g), dim3(512), 0, st, a); \
          else hipLaunchKernelGGL((conv_fwd_pers_kernel<64, 3, 0, T, SPL_>), dim3(g), dim3(512), 0, st, a); \
        } \
      } while (0)
      if (f32_split() && psplit_ok(a) && has_split_room(a)) {
        const bool tall = psplit_tall(a);
        const bool wide = psplit_wide();
        const bool inc = psplit_inc();
        // f16 x3 planes instead (presplit_h) on the default (incremental, wide) forms
        const bool h16 = f32_h16() && inc && wide;
        // the producer's pair image (the conv's scale from the producer's bound)
        const bool pair = h16 && a.xpair && a.xbound && !a.escale && !(g_stamps && getenv("DGVCC_PSPLIT_STAMP"));
        FwdArgs ah = a;
        if (pair) ah.xamax = a.xbound;
        const unsigned short* wsp = h16 ? presplit_h(ah, st) : presplit(a, st);
        if (!wsp) return DG_ERR_HIP;
        const int bn2 = f32_pers_bn(a.Cout);
        const unsigned g2 = (unsigned)std::min<long long>((long long)dg_cdiv(M, psplit_tile_px(a)) * (a.Cout / bn2),
                                                          persist_grid());
        const char* wspc = (const char*)wsp;
        FwdArgs ap = a;
        {
          const char* e = getenv("DGVCC_PSPLIT_ORDER");
          ap.tile_order = (e && e[0] == '1') ? 1 : 0;
        }
        // f16 x3: the pixel operand split once into the workspace after the filter planes (SCH 8)
        bool xs = false;
        if (pair) {
          ap.x = a.xpair;
          ap.ldx = a.C;
          xs = true;
        } else if (h16 && psplit_xs(a, bn2) && !a.escale && a.ldx % 4 == 0 && !(g_stamps && getenv("DGVCC_PSPLIT_STAMP"))) {
          const long long off = xsplit_off(presplit_h_bytes(a));
          if (a.wsplit_bytes >= off + xsplit_bytes(a)) {
            const long long KTh = (long long)a.R * a.S * (a.C / 32);
            const float* hsx = (const float*)((const char*)wsp + (long long)a.Cout * KTh * 128) + a.Cout;
            unsigned char* xsb = (unsigned char*)a.wsplit + off;
            const long long n8 = M * (a.C / 8);
            hipLaunchKernelGGL(split_x_h_kernel, dim3((unsigned)std::min<long long>(dg_cdiv(n8, 256), 16384)), dim3(256),
                               0, st, (const float*)a.x, a.ldx, M, a.C, hsx, xsb);
            DG_CHECK_LAUNCH();
            ap.x = (const char*)xsb;
            ap.ldx = a.C;
            xs = true;
          }
        }
#define PSPLIT_LAUNCH(EPI_)                                                                                    \
  do {                                                                                                         \
    if (h16 && xs) {                                                                                           \
      if (bn2 == 256) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, EPI_, 1, 1, 0, 1, 0, 8>), dim3(g2), dim3(512), 0, st, ap, wspc); \
      else hipLaunchKernelGGL((conv_fwd_psplit_kernel<128, 2, EPI_, 1, 1, 0, 1, 0, 8>), dim3(g2), dim3(512), 0, st, ap, wspc); \
    } else if (h16) {                                                                                          \
      if (bn2 == 256) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, EPI_, 1, 1, 0, 1>), dim3(g2), dim3(512), 0, st, ap, wspc); \
      else hipLaunchKernelGGL((conv_fwd_psplit_kernel<128, 2, EPI_, 1, 1, 0, 1>), dim3(g2), dim3(512), 0, st, ap, wspc); \
    } else if (bn2 == 256) {                                                                                   \
      if (inc) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, EPI_>), dim3(g2), dim3(512), 0, st, ap, wspc); \
      else hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, EPI_, 1, 0>), dim3(g2), dim3(512), 0, st, ap, wspc); \
    } else if (wide) {                                                                                         \
      if (inc) hipLaunchKernelGGL((conv_fwd_psplit_kernel<128, 2, EPI_>), dim3(g2), dim3(512), 0, st, ap, wspc); \
      else hipLaunchKernelGGL((conv_fwd_psplit_kernel<128, 2, EPI_, 1, 0>), dim3(g2), dim3(512), 0, st, ap, wspc); \
    } else hipLaunchKernelGGL((conv_fwd_psplit_kernel<128, 3, EPI_, 0>), dim3(g2), dim3(512), 0, st, ap, wspc);  \
  } while (0)
        if (a.escale) PSPLIT_LAUNCH(3);
        else if (h16 && tall && g_stamps && getenv("DGVCC_PSPLIT_STAMP") &&
                 (long long)g2 * 8 * 8 * 8 <= g_stamp_bytes) {  // diagnostic stamp build (tools/stamp_psplit.py)
          ap.stamps = g_stamps;
          const int sch = psplit_sch();
          if (sch == 5 && a.R * a.S * (a.C / 32) >= 2) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1, 1, 5>), dim3(g2), dim3(512), 0, st, ap, wspc);
          else if (sch == 4) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1, 1, 4>), dim3(g2), dim3(512), 0, st, ap, wspc);
          else if (sch == 3) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1, 1, 3>), dim3(g2), dim3(512), 0, st, ap, wspc);
          else if (sch == 2) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1, 1, 2>), dim3(g2), dim3(512), 0, st, ap, wspc);
          else if (sch == 1) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1, 1, 1>), dim3(g2), dim3(512), 0, st, ap, wspc);
          else hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1, 1>), dim3(g2), dim3(512), 0, st, ap, wspc);
        } else if (h16 && tall && xs) {
          hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1, 0, 8>), dim3(g2), dim3(512), 0, st, ap, wspc);
        } else if (h16 && tall) {
          const int sch = psplit_sch();
          if (sch == 9) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1, 0, 9>), dim3(g2), dim3(512), 0, st, ap, wspc);
          else if (sch == 6) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1, 0, 6>), dim3(g2), dim3(512), 0, st, ap, wspc);
          else if (sch == 7) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1, 0, 7>), dim3(g2), dim3(512), 0, st, ap, wspc);
          else if (sch == 5 && a.R * a.S * (a.C / 32) >= 2) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1, 0, 5>), dim3(g2), dim3(512), 0, st, ap, wspc);
          else if (sch == 4) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1, 0, 4>), dim3(g2), dim3(512), 0, st, ap, wspc);
          else if (sch == 3) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1, 0, 3>), dim3(g2), dim3(512), 0, st, ap, wspc);
          else if (sch == 2) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1, 0, 2>), dim3(g2), dim3(512), 0, st, ap, wspc);
          else if (sch == 1) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1, 0, 1>), dim3(g2), dim3(512), 0, st, ap, wspc);
          else hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1, 1>), dim3(g2), dim3(512), 0, st, ap, wspc);
        }
        else if (tall) hipLaunchKernelGGL((conv_fwd_psplit_kernel<256, 2, 0, 1, 1, 1>), dim3(g2), dim3(512), 0, st, ap, wspc);
        else PSPLIT_LAUNCH(0);
#undef PSPLIT_LAUNCH
      } else if (f32_split()) F32_PERS(1);
      else F32_PERS(0);
#undef F32_PERS
      DG_CHECK_LAUNCH();
      return DG_OK;
    }
  }
  const int npx = dg_cdiv(M, 128);
  if (a.Cout % 128 == 0) {
    const int nco = a.Cout / 128;
    hipLaunchKernelGGL((conv_fwd_kernel<T, 128, 128>), dim3(npx * nco), dim3(NT), 0, st, a);
  } else {
    const int nco = a.Cout / 64;
    hipLaunchKernelGGL((conv_fwd_kernel<T, 64, 128>), dim3(npx * nco), dim3(NT), 0, st, a);
  }
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// ---------------------------------------------------------------------------
// weight gradient: split-K over pixels into f32 slabs, then a deterministic
// reduce that also transposes to torch's [Cout][C][R][S] layout.
// ---------------------------------------------------------------------------
struct WgPlan { int splits, pps; };

struct WgArgs {
  const char* x; long long ldx; int N, H, W, C;
  const char* dy; long long lddy; int Cout, R, S, pad;
  float* slab;         // [splits][Cout][R*S*C]
  int splits, pps;     // pixels per split (multiple of BKP)
  int stride, P, Q;    // output grid of dy (stride 1: P = H, Q = W)
  int whole_x;         // 1: descriptor over the whole x (strided convs)
  int pad_ok = 0;      // 1: the plan may be the padded 9-tap kernel's (dg_conv_wgrad)
  int band = 0;        // > 0: the 9-tap wgrad walks its K-steps in bands of this many image rows
  // f32 f16 x3 arithmetic: max |x| and max |dy| as float bits (device words)
  const unsigned* xam = nullptr;
  const unsigned* dyam = nullptr;
};

template <typename T> struct WgCfg;
template <> struct WgCfg<bf16> { static constexpr int BKP = 64, PAD = 32; };
template <> struct WgCfg<f16> { static constexpr int BKP = 64, PAD = 32; };
template <> struct WgCfg<float> { static constexpr int BKP = 32, PAD = 64; };

// SPL = 1 (T = float only): the exact 3-way bf16 split (dg_common.h split3_8); one
// 32-pixel K-step is one 16x16x32 block, lane group g taking pixel rows 4m + g (m < 8),
// conflict-free as the f32 reads below.
template <typename T, int BCO, int BC, int SPL = 0>
__global__ __launch_bounds__(NT, 2) void conv_wgrad_kernel(WgArgs a) {
  constexpr int BKP = WgCfg<T>::BKP;
  constexpr int EPC = 16 / (int)sizeof(T);
  constexpr int ROWA = BCO * (int)sizeof(T) + WgCfg<T>::PAD;  // bytes per LDS row (dY tile)
  constexpr int ROWB = BC * (int)sizeof(T) + WgCfg<T>::PAD;   // bytes per LDS row (X tile)
  constexpr int CPRA = BCO / EPC, CPRB = BC / EPC;            // 16-B chunks per row
  constexpr int AR = BKP * CPRA / NT, BR = BKP * CPRB / NT;   // chunks per thread
  constexpr int TILE_BYTES = BKP * (ROWA + ROWB);
  constexpr int TI = BCO / 32, TJ = BC / 32;
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE_BYTES];

  const int HW = a.H * a.W;
  const int PQ = a.P * a.Q;
  const int M = a.N * PQ;
  const int RS = a.R * a.S;
  const int nco = a.Cout / BCO, ncb = a.C / BC;
  const int tiles = nco * ncb * RS;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / tiles;
  int t = bid - split * tiles;
  const int cot = t % nco; t /= nco;
  const int cbt = t % ncb;
  const int rs = t / ncb;
  const int co0 = cot * BCO, c0 = cbt * BC;
  const int r = rs / a.S, s = rs - r * a.S;
  const int dh = r - a.pad, dw = s - a.pad;
  const int kbeg = split * a.pps;
  const int kend = min(M, kbeg + a.pps);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

  // descriptors: dY over [kbeg, kend), X over the shifted window
  const unsigned dy_bytes = (unsigned)(((long long)(kend - kbeg - 1) * a.lddy + a.Cout) * sizeof(T));
  __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.dy + (long long)kbeg * a.lddy * sizeof(T)), 0, dy_bytes, 0x00020000);
  const int halo = a.pad * (a.W + 1);
  const int xlo = a.whole_x ? 0 : max(0, kbeg - halo);
  const int xhi = a.whole_x ? a.N * HW : min(M, kend + halo);
  const unsigned x_bytes = (unsigned)(((long long)(xhi - xlo - 1) * a.ldx + a.C) * sizeof(T));
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.x + (long long)xlo * a.ldx * sizeof(T)), 0, x_bytes, 0x00020000);

  u4v ra[AR], rb[BR];
  // (n, p, q) of each X row's output pixel, advanced by BKP per K-step: the per-step integer
  // divisions (3 per row) had made non-MFMA VALU instructions 2x the MFMA count (PMC)
  int cn[BR], cp[BR], cq[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int px = kbeg + (tid + NT * i) / CPRB;
    cn[i] = px / PQ;
    const int rem = px - cn[i] * PQ;
    cp[i] = rem / a.Q;
    cq[i] = rem - cp[i] * a.Q;
  }
  auto gload = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int idx = tid + NT * i;
      const int row = idx / CPRA, ch = idx % CPRA;
      const int px = k0 + row;
      const unsigned off = (px < kend)
          ? (unsigned)(((long long)(px - kbeg) * a.lddy + co0 + ch * EPC) * (long long)sizeof(T)) : 0xFFFFFFF0u;
      ra[i] = bload(dyr, off);
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int idx = tid + NT * i;
      const int row = idx / CPRB, ch = idx % CPRB;
      const int px = k0 + row;
      const int h = cp[i] * a.stride + dh, ww = cq[i] * a.stride + dw;
      const bool ok = px < kend && (unsigned)h < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
      const long long pin = (long long)cn[i] * HW + (long long)h * a.W + ww - xlo;
      const unsigned off = ok ? (unsigned)((pin * a.ldx + c0 + ch * EPC) * (long long)sizeof(T)) : 0xFFFFFFF0u;
      rb[i] = bload(xr, off);
      cq[i] += BKP;  // next K-step's pixel
      while (cq[i] >= a.Q) {
        cq[i] -= a.Q;
        if (++cp[i] == a.P) { cp[i] = 0; ++cn[i]; }
      }
    }
  };
  auto swrite = [&](int buf) __attribute__((always_inline)) {
    char* As = smem + buf * TILE_BYTES;
    char* Bs = As + BKP * ROWA;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int idx = tid + NT * i;
      *(u4v*)(As + (idx / CPRA) * ROWA + (idx % CPRA) * 16) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int idx = tid + NT * i;
      *(u4v*)(Bs + (idx / CPRB) * ROWB + (idx % CPRB) * 16) = rb[i];
    }
  };

  f4v acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  const int wco = (wid >> 1) * (BCO / 2), wc = (wid & 1) * (BC / 2);
  const int g = lane >> 4;

  const int nkt = (kend - kbeg + BKP - 1) / BKP;
  gload(kbeg);
  swrite(0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) gload(kbeg + (kt + 1) * BKP);
    const char* As = smem + cur * TILE_BYTES;
    const char* Bs = As + BKP * ROWA;
    if constexpr (Is16<T>::value) {
      // ds_read_b64_tr_b16: lane 4q+p of each 16-lane group supplies row q,
      // columns 4p..4p+3; lane i receives column i of the 4 rows.  The logical
      // k = 8g + j maps to physical pixel row 4g + (j&3) + 16*(j>>2) for both
      // operands (conflict-free: 8 consecutive rows per half-wave, row pitch
      // = 8 dwords mod 64).
      const int q = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
      for (int ks = 0; ks < BKP / 32; ++ks) {
        const int r1 = 32 * ks + 4 * g + q, r2 = r1 + 16;
        s8v af[TI], bfv[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const int col = (wco + 16 * i + 4 * p) * 2;
          s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DG_LDS s4v*)(As + r1 * ROWA + col));
          s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DG_LDS s4v*)(As + r2 * ROWA + col));
          af[i] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int col = (wc + 16 * j + 4 * p) * 2;
          s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DG_LDS s4v*)(Bs + r1 * ROWB + col));
          s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DG_LDS s4v*)(Bs + r2 * ROWB + col));
          bfv[j] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = mfma16x16x32<T>(af[i], bfv[j], acc[i][j]);
      }
    } else if constexpr (SPL) {
      static_assert(BKP == 32, "one 16x16x32 block per K-step");
      const int fcol = lane & 15;
      auto frag = [&](const char* base, int rowb, int col, s8v& h0, s8v& h1, s8v& h2) __attribute__((always_inline)) {
        u4v x0, x1;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          x0[m] = *(const unsigned*)(base + (4 * m + g) * rowb + col * 4);
          x1[m] = *(const unsigned*)(base + (4 * m + 16 + g) * rowb + col * 4);
        }
        split3_8_rn(x0, x1, h0, h1, h2);
      };
      s8v bh[TJ][3];
#pragma unroll
      for (int j = 0; j < TJ; ++j) frag(Bs, ROWB, wc + 16 * j + fcol, bh[j][0], bh[j][1], bh[j][2]);
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        s8v ah[3];
        frag(As, ROWA, wco + 16 * i + fcol, ah[0], ah[1], ah[2]);
        constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
        for (int q = 0; q < 6; ++q)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[PA[q]], bh[j][PB[q]], acc[i][j], 0, 0, 0);
      }
    } else {
      const int fcol = lane & 15;
#pragma unroll
      for (int ks = 0; ks < BKP / 4; ++ks) {
        const int row = 4 * ks + g;
        float af[TI], bfv[TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) af[i] = *(const float*)(As + row * ROWA + (wco + 16 * i + fcol) * 4);
#pragma unroll
        for (int j = 0; j < TJ; ++j) bfv[j] = *(const float*)(Bs + row * ROWB + (wc + 16 * j + fcol) * 4);
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfv[j], acc[i][j], 0, 0, 0);
      }
    }
    if (kt + 1 < nkt) swrite(cur ^ 1);
    __syncthreads();
  }

  // slab[split][co][rs*C + c]; lane holds column c, rows co = 4g + r
  const long long ldk = (long long)RS * a.C;
  float* out = a.slab + (long long)split * a.Cout * ldk;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int c = c0 + wc + 16 * j + (lane & 15);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int co = co0 + wco + 16 * i + 4 * g + rr;
        out[co * ldk + rs * a.C + c] = acc[i][j][rr];
      }
    }
}

// f32 weight gradient on the bf16 matrix cores (split math), one block per CU: 8 waves
// (WCO x 8/WCO over the BCO x BC tile of one (r,s) tap), K = 32 pixels per step.  The f32
// pixel rows of dY and X are loaded to registers (one step ahead), split ONCE per block
// (dg_common.h: x = h0 + h1 + h2 exactly) and stored as three bf16 planes [pixel][channel];
// fragments are read transposed with ds_read_b64_tr_b16 as in the bf16 kernel (logical
// k = 8g + j -> pixel row 4g + (j & 3) + 16 (j >> 2), both operands), six MFMA products
// per 16x16x32 block.  The per-wave fragment split (conv_wgrad_kernel SPL = 1) did 4x the
// split work of this per-block one.
// HM = 1: the f16 x3 arithmetic as conv_wgrad_split3_kernel's.
template <int BCO, int BC, int WCO, int NTH = 512, int HM = 0>
__global__ __launch_bounds__(NTH, 512 / NTH) void conv_wgrad_split_kernel(WgArgs a) {
  constexpr int BKP = 32;
  constexpr int ROWA = BCO * 2 + 32, ROWB = BC * 2 + 32;  // bytes per bf16 plane row
  constexpr int PA = BKP * ROWA, PB = BKP * ROWB;          // bytes per plane
  constexpr int NPL = HM ? 2 : 3;
  constexpr int TILE = NPL * (PA + PB);
  constexpr int CPRA = BCO / 4, CPRB = BC / 4;             // 16-B f32 chunks per pixel row
  constexpr int AR = BKP * CPRA / NTH, BR = BKP * CPRB / NTH;
  constexpr int WC = NTH / 64 / WCO;
  constexpr int TI = BCO / WCO / 16, TJ = BC / WC / 16;
  static_assert(AR >= 1 && BR >= 1 && TI >= 1 && TJ >= 1, "tile too small for the block");
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE];

  const int HW = a.H * a.W;
  const int PQ = a.P * a.Q;
  const int M = a.N * PQ;
  const int RS = a.R * a.S;
  const int nco = a.Cout / BCO, ncb = a.C / BC;
  const int tiles = nco * ncb * RS;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / tiles;
  int t = bid - split * tiles;
  const int cot = t % nco; t /= nco;
  const int cbt = t % ncb;
  const int rs = t / ncb;
  const int co0 = cot * BCO, c0 = cbt * BC;
  const int r = rs / a.S, s = rs - r * a.S;
  const int dh = r - a.pad, dw = s - a.pad;
  const int kbeg = split * a.pps;
  const int kend = min(M, kbeg + a.pps);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // HM: per-channel power-of-two scales of this thread's 4 dY and 4 X channels (its 16-byte chunks keep
  // their channels over every K-step: NTH is a multiple of both chunk counts per row)
  static_assert(NTH % CPRA == 0 && NTH % CPRB == 0, "a thread's chunks must keep their channels");
  f4v hsdy = f4v{1.f, 1.f, 1.f, 1.f}, hsx = f4v{1.f, 1.f, 1.f, 1.f};
  if constexpr (HM) {
    int e4[4];
    chan_h16_scales(a.dyam, co0 + (tid % CPRA) * 4, e4, hsdy);
    chan_h16_scales(a.xam, c0 + (tid % CPRB) * 4, e4, hsx);
  }

  const unsigned dy_bytes = (unsigned)(((long long)(kend - kbeg - 1) * a.lddy + a.Cout) * 4);
  __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.dy + (long long)kbeg * a.lddy * 4), 0, dy_bytes, 0x00020000);
  const int halo = a.pad * (a.W + 1);
  const int xlo = a.whole_x ? 0 : max(0, kbeg - halo);
  const int xhi = a.whole_x ? a.N * HW : min(M, kend + halo);
  const unsigned x_bytes = (unsigned)(((long long)(xhi - xlo - 1) * a.ldx + a.C) * 4);
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.x + (long long)xlo * a.ldx * 4), 0, x_bytes, 0x00020000);

  u4v ra[AR], rb[BR];
  int cn[BR], cp[BR], cq[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int px = kbeg + (tid + NTH * i) / CPRB;
    cn[i] = px / PQ;
    const int rem = px - cn[i] * PQ;
    cp[i] = rem / a.Q;
    cq[i] = rem - cp[i] * a.Q;
  }
  auto gload = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int idx = tid + NTH * i;
      const int row = idx / CPRA, ch = idx % CPRA;
      const int px = k0 + row;
      const unsigned off = (px < kend) ? (unsigned)(((long long)(px - kbeg) * a.lddy + co0 + ch * 4) * 4) : 0xFFFFFFF0u;
      ra[i] = bload(dyr, off);
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int idx = tid + NTH * i;
      const int row = idx / CPRB, ch = idx % CPRB;
      const int px = k0 + row;
      const int h = cp[i] * a.stride + dh, ww = cq[i] * a.stride + dw;
      const bool ok = px < kend && (unsigned)h < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
      const long long pin = (long long)cn[i] * HW + (long long)h * a.W + ww - xlo;
      const unsigned off = ok ? (unsigned)((pin * a.ldx + c0 + ch * 4) * 4) : 0xFFFFFFF0u;
      rb[i] = bload(xr, off);
      cq[i] += BKP;
      while (cq[i] >= a.Q) {
        cq[i] -= a.Q;
        if (++cp[i] == a.P) { cp[i] = 0; ++cn[i]; }
      }
    }
  };
  auto swrite = [&](int buf) __attribute__((always_inline)) {
    char* As = smem + buf * TILE;
    char* Bs = As + NPL * PA;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int idx = tid + NTH * i;
      const int o = (idx / CPRA) * ROWA + (idx % CPRA) * 8;
      if constexpr (HM) {
        u2v h0, h1;
        split2h_4v(ra[i], hsdy, h0, h1);
        *(u2v*)(As + o) = h0;
        *(u2v*)(As + PA + o) = h1;
      } else {
        u2v h0, h1, h2;
        split3_4_rn(ra[i], h0, h1, h2);
        *(u2v*)(As + o) = h0;
        *(u2v*)(As + PA + o) = h1;
        *(u2v*)(As + 2 * PA + o) = h2;
      }
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int idx = tid + NTH * i;
      const int o = (idx / CPRB) * ROWB + (idx % CPRB) * 8;
      if constexpr (HM) {
        u2v h0, h1;
        split2h_4v(rb[i], hsx, h0, h1);
        *(u2v*)(Bs + o) = h0;
        *(u2v*)(Bs + PB + o) = h1;
      } else {
        u2v h0, h1, h2;
        split3_4_rn(rb[i], h0, h1, h2);
        *(u2v*)(Bs + o) = h0;
        *(u2v*)(Bs + PB + o) = h1;
        *(u2v*)(Bs + 2 * PB + o) = h2;
      }
    }
  };

  f4v acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  const int wco = (wid / WC) * (BCO / WCO), wc = (wid % WC) * (BC / WC);
  const int g = lane >> 4;
  const int q = (lane & 15) >> 2, p4 = lane & 3;
  const int r1 = 4 * g + q, r2 = r1 + 16;

  const int nkt = (kend - kbeg + BKP - 1) / BKP;
  gload(kbeg);
  swrite(0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) gload(kbeg + (kt + 1) * BKP);
    const char* As = smem + cur * TILE;
    const char* Bs = As + NPL * PA;
    s8v bh[TJ][NPL];
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int col = (wc + 16 * j + 4 * p4) * 2;
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) {
        const char* b = Bs + pl * PB;
        s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DG_LDS s4v*)(b + r1 * ROWB + col));
        s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DG_LDS s4v*)(b + r2 * ROWB + col));
        bh[j][pl] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
    }
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int col = (wco + 16 * i + 4 * p4) * 2;
      s8v ah[NPL];
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) {
        const char* b = As + pl * PA;
        s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DG_LDS s4v*)(b + r1 * ROWA + col));
        s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DG_LDS s4v*)(b + r2 * ROWA + col));
        ah[pl] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      if constexpr (HM) {
        constexpr int PA3[3] = {1, 0, 0}, PB3[3] = {0, 1, 0};
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8v, ah[PA3[u]]),
                                                               __builtin_bit_cast(h8v, bh[j][PB3[u]]), acc[i][j], 0, 0, 0);
      } else {
        constexpr int PA6[6] = {2, 1, 0, 1, 0, 0}, PB6[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
        for (int u = 0; u < 6; ++u)
#pragma unroll
          for (int j = 0; j < TJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[PA6[u]], bh[j][PB6[u]], acc[i][j], 0, 0, 0);
      }
      // the next step's split + LDS stores between the MFMA blocks (the other buffer was last
      // read before the previous barrier), so its VALU/LDS work overlaps this step's MFMAs
      if (NTH == 512 && i == (TI - 1) / 2 && kt + 1 < nkt) swrite(cur ^ 1);
    }
    if (NTH != 512 && kt + 1 < nkt) swrite(cur ^ 1);  // two blocks per CU overlap each other instead
    __syncthreads();
  }

  const long long ldk = (long long)RS * a.C;
  float* out = a.slab + (long long)split * a.Cout * ldk;
  // HM: back by 2^-(e_dy[co] + e_x[c]), applied to the value (exact unless the result itself leaves
  // f32's range, as an f32 product would)
  int ecol[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) ecol[j] = HM ? h16_exp(__uint_as_float(a.xam[1 + c0 + wc + 16 * j + (lane & 15)])) : 0;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int co = co0 + wco + 16 * i + 4 * g + rr;
      const int erow = HM ? h16_exp(__uint_as_float(a.dyam[1 + co])) : 0;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int c = c0 + wc + 16 * j + (lane & 15);
        out[co * ldk + rs * a.C + c] = HM ? ldexpf(acc[i][j][rr], -(erow + ecol[j])) : acc[i][j][rr];
      }
    }
}

// f32 weight gradient of a 3x3 / stride-1 / pad-1 conv on the split math with the three taps of
// one kernel row sharing their operands (the bf16 conv_wgrad9_kernel's idea on
// conv_wgrad_split_kernel's split-once-per-block staging): a K-step is 32 consecutive pixels of
// one image row (W % 32 == 0); dY[32 px][BCO] and the input strip X[34 px][BC] of image row
// p + r - 1 (columns q0 - 1 .. q0 + 32) are split once into bf16 planes, and the taps s = 0, 1, 2
// read the strip at row offsets s.  Per staged value 3x the MFMA work of the per-tap kernel.
// 64 x 64 (x 3 taps): 4 waves of 32 x 32, two blocks per CU (the per-tap kernel's 64-wide tiles
// were bound by the split and LDS-store work, ~30% MFMA-busy); 128 x 128: 8 waves of 64 x 32,
// one block per CU.
// NR = 3 (the 64-channel layers, 8 waves of 32 x 16 x 9 taps): a block owns all three kernel rows,
// staging the dY rows once and the three X strips of image rows p - 1, p, p + 1 per K-step, instead
// of three blocks (one per kernel row) each staging and splitting the same dY rows: 33% less split
// and staging work per MFMA (DGVCC_WGRAD_SPLIT9=0: the 64 x 64 x 3-tap blocks).
// HM = 1: the f16 x3 arithmetic (dg_common.h): dY and X scaled by their tensors' powers of two
// (a.dyam / a.xam) and split into two f16 planes each, three MFMAs per block, the slab written
// back at 2^-(e_dy + e_x).
template <int BCO, int BC, int WCO, int NTH, int SWP = 0, int NR = 1, int HM = 0>
__global__ __launch_bounds__(NTH, 512 / NTH) void conv_wgrad_split3_kernel(WgArgs a) {
  static_assert(NR == 1 || NR == 3, "one kernel row per block, or all three");
  constexpr int BKP = 32, XR = BKP + 2;
  constexpr int ROWA = BCO * 2 + 32, ROWB = BC * 2 + 32;  // bytes per bf16 plane row
  constexpr int PA = BKP * ROWA, PB = XR * ROWB;           // bytes per plane
  constexpr int NPL = HM ? 2 : 3;  // planes per operand
  constexpr int TILE = NPL * (PA + NR * PB);
  constexpr int CPRA = BCO / 4, CPRB = BC / 4;             // 16-B f32 chunks per pixel row
  constexpr int AR = BKP * CPRA / NTH, BR = (NR * XR * CPRB + NTH - 1) / NTH;
  constexpr int WC = NTH / 64 / WCO;
  constexpr int TI = BCO / WCO / 16, TJ = BC / WC / 16;
  static_assert(AR * NTH == BKP * CPRA && TI >= 1 && TJ >= 1, "tile / block mismatch");
  __shared__ __attribute__((aligned(16))) char smem[2 * TILE];

  const int HW = a.H * a.W;
  const int M = a.N * HW;
  const int nco = a.Cout / BCO, ncb = a.C / BC;
  const int tiles = nco * ncb * (NR == 3 ? 1 : 3);
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / tiles;
  int t = bid - split * tiles;
  const int cot = t % nco; t /= nco;
  const int cbt = t % ncb;
  const int r = NR == 3 ? 0 : t / ncb;  // kernel row (NR = 1)
  const int co0 = cot * BCO, c0 = cbt * BC;
  const int dh = r - 1;
  const int kbeg = split * a.pps;
  const int kend = min(M, kbeg + a.pps);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // HM: per-channel power-of-two scales of this thread's 4 dY and 4 X channels (its 16-byte chunks keep
  // their channels over every K-step: NTH is a multiple of both chunk counts per row)
  static_assert(NTH % CPRA == 0 && NTH % CPRB == 0, "a thread's chunks must keep their channels");
  f4v hsdy = f4v{1.f, 1.f, 1.f, 1.f}, hsx = f4v{1.f, 1.f, 1.f, 1.f};
  if constexpr (HM) {
    int e4[4];
    chan_h16_scales(a.dyam, co0 + (tid % CPRA) * 4, e4, hsdy);
    chan_h16_scales(a.xam, c0 + (tid % CPRB) * 4, e4, hsx);
  }

  const unsigned dy_bytes = (unsigned)(((long long)(kend - kbeg - 1) * a.lddy + a.Cout) * 4);
  __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.dy + (long long)kbeg * a.lddy * 4), 0, dy_bytes, 0x00020000);
  const int halo = a.W + 1;
  const int xlo = max(0, kbeg - halo);
  const int xhi = min(M, kend + halo);
  const unsigned x_bytes = (unsigned)(((long long)(xhi - xlo - 1) * a.ldx + a.C) * 4);
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.x + (long long)xlo * a.ldx * 4), 0, x_bytes, 0x00020000);

  // pixel coordinates of the current K-step's first pixel (uniform over the block)
  int sn = kbeg / HW, sp = (kbeg - sn * HW) / a.W, sq = kbeg - sn * HW - sp * a.W;
  u4v ra[AR], rb[BR];
  // per-lane parts of the load offsets, fixed over the K loop: 32-bit byte offsets (the buffer windows
  // are < 2^31 bytes, checked by the launcher) with the uniform per-K-step part added in the loop, and
  // an unconditional select for the out-of-image taps (no 64-bit multiplies, no exec-mask branches)
  unsigned aoff[AR], boff[BR];
  int brow[BR], bstrip[BR];
  bool bval[BR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int idx = tid + NTH * i;
    aoff[i] = (unsigned)((idx / CPRA) * a.lddy + co0 + (idx % CPRA) * 4) * 4u;
  }
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int idx = tid + NTH * i;
    const int strip = NR == 3 ? idx / (XR * CPRB) : 0, sidx = idx - strip * (XR * CPRB);
    bstrip[i] = strip;
    brow[i] = sidx / CPRB;
    bval[i] = idx < NR * XR * CPRB;
    boff[i] = (unsigned)(brow[i] * a.ldx + c0 + (sidx % CPRB) * 4) * 4u;
  }
  const unsigned ldx4 = (unsigned)a.ldx * 4u, lddy4 = (unsigned)a.lddy * 4u;
  auto gload = [&](int k0) __attribute__((always_inline)) {
    const unsigned abase = (unsigned)(k0 - kbeg) * lddy4;
#pragma unroll
    for (int i = 0; i < AR; ++i) ra[i] = bload(dyr, abase + aoff[i]);
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int h = sp + (NR == 3 ? bstrip[i] - 1 : dh);
      const bool ok = bval[i] && (unsigned)h < (unsigned)a.H && (unsigned)(sq - 1 + brow[i]) < (unsigned)a.W;
      // pixel of strip row 0 (column sq - 1) relative to the window start, times the pixel stride
      const unsigned sbase = (unsigned)(sn * HW + h * a.W + sq - 1 - xlo) * ldx4;
      rb[i] = bload(xr, ok ? sbase + boff[i] : 0xFFFFFFF0u);
    }
    sq += BKP;
    if (sq >= a.W) {
      sq = 0;
      if (++sp == a.H) { sp = 0; ++sn; }
    }
  };
  auto swrite = [&](int buf, int part = 3) __attribute__((always_inline)) {
    char* As = smem + buf * TILE;
    char* Bs = As + NPL * PA;
#pragma unroll
    for (int i = 0; i < AR * (part & 1); ++i) {
      const int idx = tid + NTH * i;
      const int o = (idx / CPRA) * ROWA + (idx % CPRA) * 8;
      if constexpr (HM) {
        u2v h0, h1;
        split2h_4v(ra[i], hsdy, h0, h1);
        *(u2v*)(As + o) = h0;
        *(u2v*)(As + PA + o) = h1;
      } else {
        u2v h0, h1, h2;
        split3_4_rn(ra[i], h0, h1, h2);
        *(u2v*)(As + o) = h0;
        *(u2v*)(As + PA + o) = h1;
        *(u2v*)(As + 2 * PA + o) = h2;
      }
    }
#pragma unroll
    for (int i = 0; i < BR * ((part >> 1) & 1); ++i) {
      const int idx = tid + NTH * i;
      if (idx < NR * XR * CPRB) {
        const int strip = NR == 3 ? idx / (XR * CPRB) : 0, sidx = idx - strip * (XR * CPRB);
        const int o = strip * NPL * PB + (sidx / CPRB) * ROWB + (sidx % CPRB) * 8;
        if constexpr (HM) {
          u2v h0, h1;
          split2h_4v(rb[i], hsx, h0, h1);
          *(u2v*)(Bs + o) = h0;
          *(u2v*)(Bs + PB + o) = h1;
        } else {
          u2v h0, h1, h2;
          split3_4_rn(rb[i], h0, h1, h2);
          *(u2v*)(Bs + o) = h0;
          *(u2v*)(Bs + PB + o) = h1;
          *(u2v*)(Bs + 2 * PB + o) = h2;
        }
      }
    }
  };

  f4v acc[3 * NR][TI][TJ];
#pragma unroll
  for (int s = 0; s < 3 * NR; ++s)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[s][i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  const int wco = (wid / WC) * (BCO / WCO), wc = (wid % WC) * (BC / WC);
  const int g = lane >> 4;
  const int q = (lane & 15) >> 2, p4 = lane & 3;
  const int r1 = 4 * g + q, r2 = r1 + 16;

  const int nkt = (kend - kbeg) / BKP;
  gload(kbeg);
  swrite(0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) gload(kbeg + (kt + 1) * BKP);
    const char* As = smem + cur * TILE;
    const char* Bs = As + NPL * PA;
    s8v ah[TI][NPL];
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int col = (wco + 16 * i + 4 * p4) * 2;
#pragma unroll
      for (int pl = 0; pl < NPL; ++pl) {
        const char* b = As + pl * PA;
        s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DG_LDS s4v*)(b + r1 * ROWA + col));
        s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DG_LDS s4v*)(b + r2 * ROWA + col));
        ah[i][pl] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
    }
#pragma unroll
    for (int rs = 0; rs < 3 * NR; ++rs) {
      const int s = rs % 3;
      s8v bh[TJ][NPL];
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int col = (wc + 16 * j + 4 * p4) * 2;
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl) {
          const char* b = Bs + (rs / 3) * NPL * PB + pl * PB;
          s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DG_LDS s4v*)(b + (r1 + s) * ROWB + col));
          s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DG_LDS s4v*)(b + (r2 + s) * ROWB + col));
          bh[j][pl] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
      }
      if constexpr (HM) {
        constexpr int PA3[3] = {1, 0, 0}, PB3[3] = {0, 1, 0};
#pragma unroll
        for (int u = 0; u < 3; ++u)
#pragma unroll
          for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[rs][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                  __builtin_bit_cast(h8v, ah[i][PA3[u]]), __builtin_bit_cast(h8v, bh[j][PB3[u]]), acc[rs][i][j], 0, 0, 0);
      } else {
        constexpr int PA6[6] = {2, 1, 0, 1, 0, 0}, PB6[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
        for (int u = 0; u < 6; ++u)
#pragma unroll
          for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[rs][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i][PA6[u]], bh[j][PB6[u]], acc[rs][i][j], 0, 0, 0);
      }
      // one block per CU: the next step's split + LDS stores between the taps' MFMA blocks
      if (NTH == 512 && kt + 1 < nkt) {
        if (SWP == 0 && rs == 1) swrite(cur ^ 1);
        if (SWP == 1 && rs == 0) swrite(cur ^ 1, 1);
        if (SWP == 1 && rs == 1) swrite(cur ^ 1, 2);
        if (SWP == 2 && rs == 0) swrite(cur ^ 1);
      }
    }
    if (NTH != 512 && kt + 1 < nkt) swrite(cur ^ 1);  // two blocks per CU overlap each other instead
    __syncthreads();
  }

  const long long ldk = 9ll * a.C;
  float* out = a.slab + (long long)split * a.Cout * ldk;
  // HM: back by 2^-(e_dy[co] + e_x[c]) on the value (as conv_wgrad_split_kernel)
  int ecol[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) ecol[j] = HM ? h16_exp(__uint_as_float(a.xam[1 + c0 + wc + 16 * j + (lane & 15)])) : 0;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int co = co0 + wco + 16 * i + 4 * g + rr;
      const int erow = HM ? h16_exp(__uint_as_float(a.dyam[1 + co])) : 0;
#pragma unroll
      for (int s = 0; s < 3 * NR; ++s)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
          const int c = c0 + wc + 16 * j + (lane & 15);
          out[co * ldk + (r * 3 + s) * a.C + c] = HM ? ldexpf(acc[s][i][j][rr], -(erow + ecol[j])) : acc[s][i][j][rr];
        }
    }
}

// Split plan of conv_wgrad_split_kernel: one block per CU (256 slots), 32-pixel K-steps.
static WgPlan wgs_plan(long long M, long long tiles, long long slots = 256) {
  const long long max_split = (M + 32 * 4 - 1) / (32 * 4);
  long long splits = 1;
  double best_eff = -1.0;
  for (int rounds = 1; rounds <= 32; ++rounds) {
    long long sp = std::max(1ll, std::min(slots * rounds / tiles, max_split));
    const long long blocks = tiles * sp;
    const double eff = (double)blocks / (double)(slots * ((blocks + slots - 1) / slots));
    if (eff > best_eff + 1e-9) { best_eff = eff; splits = sp; }
    if (eff >= 0.96 || sp == max_split) break;
  }
  long long pps = (M + splits - 1) / splits;
  pps = (pps + 31) / 32 * 32;
  splits = (M + pps - 1) / pps;
  return WgPlan{(int)splits, (int)pps};
}
static bool use_wgrad_split() {  // DGVCC_WGRAD_SPLIT=0: f32 split-math wgrad on conv_wgrad_kernel SPL = 1
  const char* e = getenv("DGVCC_WGRAD_SPLIT");
  return !(e && e[0] == '0');
}
// tile (BCO x BC) and resident blocks per CU of conv_wgrad_split_kernel for a shape: 128 x 256 /
// 128 x 128 / 128 x 64 (512 threads, one block per CU), 64 x 64 (256 threads, two per CU)
static bool wgs_ok(int C, int Cout) { return use_wgrad_split() && Cout % 64 == 0 && C % 64 == 0; }
static int wgs_bco(int C, int Cout) { return Cout % 128 == 0 ? 128 : 64; }
static int wgs_bc(int C, int Cout) {
  return wgs_bco(C, Cout) == 64 ? 64 : (C % 256 == 0 ? 256 : (C % 128 == 0 ? 128 : 64));
}
static long long wgs_tiles(int C, int Cout, int RS) {
  return (long long)(Cout / wgs_bco(C, Cout)) * (C / wgs_bc(C, Cout)) * RS;
}
static long long wgs_slots(int C, int Cout) { return wgs_bco(C, Cout) == 64 ? 512 : 256; }

// conv_wgrad_split3_kernel (three taps of a kernel row share their operands) for 3x3 / pad 1 /
// stride 1 rows of W % 32 == 0; DGVCC_WGRAD_SPLIT3 = 0 off, 1 / 2 / 3 below
static int wgrad_split3_mode() {
  const char* e = getenv("DGVCC_WGRAD_SPLIT3");
  return e ? (e[0] - '0') : 3;
}
// tile side of the 3-tap kernel for a shape: 64 (64 x 64, two blocks per CU), 128 (128 x 128, one
// block per CU), 0 = not served.  Mode 1: 64-channel shapes; 2: 64-tiles for every C % 64 == 0
// shape; 3 (default): mode 1 + 128-tiles for C, Cout % 128 == 0 (fp32 final step 454 -> 427 ms
// against mode 1, same box, profiles/round2f/wgrad3_ab.txt)
static int wgs3_tile(int C, int Cout, int R, int S, int W) {
  const int m = wgrad_split3_mode();
  if (!use_wgrad_split() || m == 0 || R != 3 || S != 3 || W % 32 != 0 || C % 64 != 0 || Cout % 64 != 0) return 0;
  if (C == 64 || Cout == 64 || m == 2) return 64;
  if (m == 3 && C % 128 == 0 && Cout % 128 == 0) return 128;
  return 0;
}
static bool wgs3_shape_ok(int C, int Cout, int R, int S, int W) { return wgs3_tile(C, Cout, R, S, W) != 0; }
static long long wgs3_tiles(int C, int Cout, int b) { return (long long)(Cout / b) * (C / b) * 3; }
// the 64-tile layers on the 9-tap (all three kernel rows per block) form: DGVCC_WGRAD_SPLIT9=0 off
static bool wgs9_on(int b3) {
  if (b3 != 64) return false;
  const char* e = getenv("DGVCC_WGRAD_SPLIT9");
  return !(e && e[0] == '0');
}
static long long wgs9_tiles(int C, int Cout) { return (long long)(Cout / 64) * (C / 64); }
static long long wgs3_slots(int b) { return b == 64 ? 512 : 256; }

__global__ void wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int Cout, int C, int RS,
                                    float* __restrict__ dw, int accumulate) {
  const long long total = (long long)Cout * C * RS;
  const long long ldk = (long long)RS * C;
  for (long long o = blockIdx.x * (long long)blockDim.x + threadIdx.x; o < total;
       o += (long long)gridDim.x * blockDim.x) {
    // o indexes the slab layout [co][rs][c] (coalesced reads)
    const int c = (int)(o % C);
    const long long t = o / C;
    const int rs = (int)(t % RS);
    const int co = (int)(t / RS);
    // 8 independent loads in flight per thread (fixed pairing order: deterministic)
    const long long sstr = (long long)Cout * ldk;
    float acc8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int sp = 0;
    for (; sp + 8 <= splits; sp += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) acc8[u] += slab[(long long)(sp + u) * sstr + o];
    }
    for (int u = 0; sp < splits; ++sp, ++u) acc8[u] += slab[(long long)sp * sstr + o];
    const float sum = ((acc8[0] + acc8[1]) + (acc8[2] + acc8[3])) + ((acc8[4] + acc8[5]) + (acc8[6] + acc8[7]));
    float* d = dw + ((long long)co * C + c) * RS + rs;
    *d = accumulate ? *d + sum : sum;
  }
}

// bf16 weight gradient, pipelined: 8 waves (2 co x 4 c) over a BCO x BC tile of
// one (r,s) tap, K = 64 pixels per step.  dY and X pixel rows are staged by
// LDS-DMA into a 3-stage ring (one raw barrier per step, counted vmcnt) and read
// transposed with ds_read_b64_tr_b16.  Rows are unpadded (DMA images are
// lane-linear); bank conflicts of the transposed reads are removed by an XOR
// swizzle of the 16-B chunk index with the row (applied on the DMA source side).
template <int CPR>
__device__ __forceinline__ int wg_swz(int r) { return CPR >= 16 ? 2 * (r & 7) : 2 * ((r >> 1) & 3); }

template <int BCO, int BC, typename T = bf16>
__global__ __launch_bounds__(512, 1) void conv_wgrad_pipe_kernel(WgArgs a) {
  constexpr int BKP = 64;
  constexpr int RA = BCO * 2, RB = BC * 2;                 // bytes per LDS row
  constexpr int CPRA = RA / 16, CPRB = RB / 16;            // 16-B chunks per row
  constexpr int RPIA = 1024 / RA, RPIB = 1024 / RB;        // rows per DMA instruction
  constexpr int AIw = BKP * RA / 1024 / 8, BIw = BKP * RB / 1024 / 8;   // DMA instr. per wave per step
  constexpr int STAGE = BKP * (RA + RB);
  constexpr int TI = BCO / 32, TJ = BC / 64;
  static_assert(AIw >= 1 && BIw >= 1, "tile too small for 8 loader waves");
  __shared__ __attribute__((aligned(1024))) char smem[PSTAGES * STAGE];

  const int HW = a.H * a.W;
  const int PQ = a.P * a.Q;
  const int M = a.N * PQ;
  const int RS = a.R * a.S;
  const int nco = a.Cout / BCO, ncb = a.C / BC;
  const int tiles = nco * ncb * RS;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / tiles;
  int t = bid - split * tiles;
  const int cot = t % nco; t /= nco;
  const int cbt = t % ncb;
  const int rs = t / ncb;
  const int co0 = cot * BCO, c0 = cbt * BC;
  const int r = rs / a.S, s = rs - r * a.S;
  const int dh = r - a.pad, dw = s - a.pad;
  const int kbeg = split * a.pps;
  const int kend = min(M, kbeg + a.pps);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);

  const unsigned dy_bytes = (unsigned)(((long long)(kend - kbeg - 1) * a.lddy + a.Cout) * 2);
  __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.dy + (long long)kbeg * a.lddy * 2), 0, dy_bytes, 0x00020000);
  const int halo = a.pad * (a.W + 1);
  const int xlo = a.whole_x ? 0 : max(0, kbeg - halo);
  const int xhi = a.whole_x ? a.N * HW : min(M, kend + halo);
  const unsigned x_bytes = (unsigned)(((long long)(xhi - xlo - 1) * a.ldx + a.C) * 2);
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.x + (long long)xlo * a.ldx * 2), 0, x_bytes, 0x00020000);

  // DMA geometry of this lane: row within the instruction and the source chunk
  const int arow = lane / CPRA, achunk = (lane % CPRA) ^ wg_swz<CPRA>(arow);
  const int brow = lane / CPRB, bchunk = (lane % CPRB) ^ wg_swz<CPRB>(brow);
  // (rows of instruction ii start at ii*RPI: RPI is a multiple of 8 or divides 8,
  //  so wg_swz(ii*RPI + row) == wg_swz(row) whenever RPI >= 8 ... handled below)
  const int nkt = (kend - kbeg + BKP - 1) / BKP;
  int bn[BIw], bp[BIw], bq[BIw];  // output-grid coordinates of this lane's X rows at the next issue
#pragma unroll
  for (int i = 0; i < BIw; ++i) {
    const int px = kbeg + (wid * BIw + i) * RPIB + brow;
    bn[i] = px / PQ;
    const int rem = px - bn[i] * PQ;
    bp[i] = rem / a.Q;
    bq[i] = rem - bp[i] * a.Q;
  }

#define WG_ISSUE(kt_, stage_) \
  do { \
    const int k0 = kbeg + (kt_) * BKP; \
    char* As = smem + (stage_) * STAGE; \
    char* Bs = As + BKP * RA; \
    _Pragma("unroll") for (int i = 0; i < AIw; ++i) { \
      const int ii = wid * AIw + i; \
      const int row = ii * RPIA + arow; \
      const int ch = (lane % CPRA) ^ wg_swz<CPRA>(row); \
      const int px = k0 + row; \
      const unsigned off = px < kend ? (unsigned)(((long long)(px - kbeg) * a.lddy + co0 + ch * 8) * 2) : 0xFFFFFFF0u; \
      lds_dma16(dyr, As + ii * 1024, off); \
    } \
    _Pragma("unroll") for (int i = 0; i < BIw; ++i) { \
      const int ii = wid * BIw + i; \
      const int row = ii * RPIB + brow; \
      const int ch = (lane % CPRB) ^ wg_swz<CPRB>(row); \
      const int px = k0 + row; \
      const int h = bp[i] * a.stride + dh, ww = bq[i] * a.stride + dw; \
      const bool ok = px < kend && (unsigned)h < (unsigned)a.H && (unsigned)ww < (unsigned)a.W; \
      const long long pin = (long long)bn[i] * HW + (long long)h * a.W + ww - xlo; \
      const unsigned off = ok ? (unsigned)((pin * a.ldx + c0 + ch * 8) * 2) : 0xFFFFFFF0u; \
      lds_dma16(xr, Bs + ii * 1024, off); \
      /* advance this row's (n, p, q) by one K-step (64 pixels): no divisions in the loop */ \
      bq[i] += BKP; \
      while (bq[i] >= a.Q) { bq[i] -= a.Q; if (++bp[i] >= a.P) { bp[i] = 0; ++bn[i]; } } \
    } \
  } while (0)
  (void)achunk; (void)bchunk;

  f4v acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  const int wco = (wid >> 2) * (BCO / 2), wc = (wid & 3) * (BC / 4);
  const int g = lane >> 4, q = (lane & 15) >> 2, p4 = lane & 3;

  WG_ISSUE(0, 0);
  if (nkt > 1) WG_ISSUE(1, 1);
  for (int kt = 0; kt < nkt; ++kt) {
    if (kt + 1 < nkt) {
      if constexpr (AIw + BIw == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else if constexpr (AIw + BIw == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else if constexpr (AIw + BIw == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if constexpr (AIw + BIw == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + 2 < nkt) WG_ISSUE(kt + 2, (kt + 2) % PSTAGES);
    const char* As = smem + (kt % PSTAGES) * STAGE;
    const char* Bs = As + BKP * RA;
#pragma unroll
    for (int ks = 0; ks < BKP / 32; ++ks) {
      const int r1 = 32 * ks + 4 * g + q, r2 = r1 + 16;
      s8v af[TI], bfv[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int cc = (wco + 16 * i) / 8 + (p4 >> 1);
        const int hb = (p4 & 1) * 8;
        s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DG_LDS s4v*)(As + r1 * RA + ((cc ^ wg_swz<CPRA>(r1)) << 4) + hb));
        s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DG_LDS s4v*)(As + r2 * RA + ((cc ^ wg_swz<CPRA>(r2)) << 4) + hb));
        af[i] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int cc = (wc + 16 * j) / 8 + (p4 >> 1);
        const int hb = (p4 & 1) * 8;
        s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DG_LDS s4v*)(Bs + r1 * RB + ((cc ^ wg_swz<CPRB>(r1)) << 4) + hb));
        s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DG_LDS s4v*)(Bs + r2 * RB + ((cc ^ wg_swz<CPRB>(r2)) << 4) + hb));
        bfv[j] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = mfma16x16x32<T>(af[i], bfv[j], acc[i][j]);
    }
  }
#undef WG_ISSUE

  const long long ldk = (long long)RS * a.C;
  float* out = a.slab + (long long)split * a.Cout * ldk;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
      const int c = c0 + wc + 16 * j + (lane & 15);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int co = co0 + wco + 16 * i + 4 * g + rr;
        out[co * ldk + rs * a.C + c] = acc[i][j][rr];
      }
    }
}

// ---------------------------------------------------------------------------
// bf16 weight gradient of a 3x3 / stride 1 / pad 1 conv with all 9 taps fused in
// one block (W % 64 == 0).  A K-step is 64 output pixels of ONE image row; the
// block stages dY[64 px][BCO] once and, per kernel row dh, the 72-pixel X strip
// [q0-4, q0+68) of image row p+dh-1 (64 channels), so every tap reads shifted
// rows of the same LDS image: 9 GEMM taps per dY tile, ~4x fewer L2->LDS bytes
// per FLOP than one-tap-per-block.  LDS-DMA 3-stage ring as conv_fwd_pipe_kernel;
// transposed fragment reads (ds_read_b64_tr_b16) on XOR-swizzled rows.
// ---------------------------------------------------------------------------
constexpr int W9_XROWS = 72;

// WT = 1 (BCO 128): wave tile 64 co x 16 c (TI 4, TJ 1) instead of 32 x 32: the 9 taps' B
// fragments are read once per 4 A fragments (fewer transposed LDS reads per MFMA).
// WT = 2 (BCO 64): wave tile 64 co x 16 c, the 8 waves split as 4 channel groups x 2 k-halves
// (wave group kh takes the 32-px k-substep kh of every K-step) and each k-half writes its own
// f32 slab split (the reduce sums 2x the splits).  The 32 co x 16 c tile of WT = 0 read 22
// transposed fragments per 18 MFMAs and left the 64-channel layer LDS-bound.
// PADK = 1 (W % 64 != 0, the 40/20-wide deep layers of 320-px crops): the K index runs over
// the zero-padded image, u = (n, p+1, q+1) in N x (H+2) x (W+2), so a K-step of 64 u may
// span rows and every shifted strip read lands on a zero pad cell exactly where the conv's
// padding is: dy rows of pad cells are zero, x rows outside the image are zero.  Costs
// (H+2)(W+2)/HW more K (10% at 40x40) instead of falling back to the per-tap kernel.
// SCH (DMA issue point of the K-step after next): 0 = right after the barrier; 2 (default) =
// after the first 32-px k-substep's MFMAs, MFMA blocks under s_setprio(1), as
// conv_fwd_pipe_kernel (A/B in one call: wgrad 881 -> 949 TF/s, 15.1 -> 14.0 ms per step).
// Measured and dropped: setprio alone (no change), priority without the moved issue (-0.7%),
// the issue split over two points of the substep loop (777 TF/s).
// INC (W % 64 == 0 path): the DMA addressing of a K-step is incremental: the step's row
// coordinates (n, p, q0) advance by 64 pixels without divisions, and each of the wave's <= 6
// pieces keeps its lane-constant byte offset (and X row), so a piece costs one scalar-offset add
// and, for X, a column test.  INC = 0 (DGVCC_WG9_INC=0) recomputes every piece each K-step.
template <int BCO, int WT = 0, int PADK = 0, int SCH = 0, typename T = bf16, int INC = 1>
__global__ __launch_bounds__(512, 1) void conv_wgrad9_kernel(WgArgs a) {
  constexpr int BKP = 64, BC = 64;
  constexpr int RA = BCO * 2, RX = BC * 2;                    // bytes per LDS row
  constexpr int CPRA = RA / 16, CPRX = RX / 16;
  constexpr int RPIA = 1024 / RA;                             // A rows per DMA instruction
  constexpr int A_INST = BKP * RA / 1024;                     // 16 (BCO 128) / 8 (BCO 64)
  constexpr int X_INST = 3 * W9_XROWS * RX / 1024;            // 27
  constexpr int N_INST = A_INST + X_INST;
  constexpr int A_BYTES = BKP * RA, X_BYTES = W9_XROWS * RX;
  constexpr int STAGE = A_BYTES + 3 * X_BYTES;
  constexpr bool WIDE = BCO == 128 && WT == 1;
  constexpr bool KH = BCO == 64 && WT == 2;
  constexpr int TI = (WIDE || KH) ? 4 : 2, TJ = (BCO == 128 && !WIDE) ? 2 : 1;  // wave tile: 16*TI co x 16*TJ c, 9 taps
  __shared__ __attribute__((aligned(1024))) char smem[PSTAGES * STAGE];

  const int HW = a.H * a.W;
  const int M = a.N * HW;
  const int nco = a.Cout / BCO, ncb = a.C / BC;
  const int tiles = nco * ncb;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / tiles;
  const int t0 = bid - split * tiles;
  const int co0 = (t0 % nco) * BCO, c0 = (t0 / nco) * BC;
  const int PW = a.W + 2, PHW = (a.H + 2) * PW;
  const int U = PADK ? a.N * PHW : M;                        // K index space
  const int kbeg = split * a.pps;
  const int kend = min(U, kbeg + a.pps);
  const int nkt = PADK ? (kend - kbeg + BKP - 1) / BKP : (kend - kbeg) / BKP;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int dylo = PADK ? 0 : kbeg, dyhi = PADK ? M : kend;
  const unsigned dy_bytes = (unsigned)(((long long)(dyhi - dylo - 1) * a.lddy + a.Cout) * 2);
  __amdgpu_buffer_rsrc_t dyr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.dy + (long long)dylo * a.lddy * 2), 0, dy_bytes, 0x00020000);
  const int halo = a.W + 8;
  const int xlo = PADK ? 0 : max(0, kbeg - halo), xhi = PADK ? M : min(M, kend + halo);
  const unsigned x_bytes = (unsigned)(((long long)(xhi - xlo - 1) * a.ldx + a.C) * 2);
  __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.x + (long long)xlo * a.ldx * 2), 0, x_bytes, 0x00020000);
  const int my_inst = (N_INST - wid + 7) / 8;                 // wave-uniform DMA count per step

  // padded index -> image pixel (or -1 on a pad cell / outside [0, U))
  auto unpad = [&](int u) -> int {
    if (u < 0 || u >= U) return -1;
    const int n = u / PHW, r = u - n * PHW;
    const int pp = r / PW, qq = r - pp * PW;
    if (pp < 1 || pp > a.H || qq < 1 || qq > a.W) return -1;
    return n * HW + (pp - 1) * a.W + (qq - 1);
  };

#define W9_ISSUE_PAD(kt_, stage_) \
  do { \
    const int u0 = kbeg + (kt_) * BKP; \
    char* As = smem + (stage_) * STAGE; \
    char* Xs = As + A_BYTES; \
    for (int ii = wid; ii < N_INST; ii += 8) { \
      if (ii < A_INST) { \
        const int row = ii * RPIA + lane / CPRA; \
        const int ch = (lane % CPRA) ^ wg_swz<CPRA>(row); \
        const int px = (u0 + row < kend) ? unpad(u0 + row) : -1; \
        lds_dma16(dyr, As + ii * 1024, px >= 0 ? (unsigned)(((long long)px * a.lddy + co0 + ch * 8) * 2) : 0xFFFFFFF0u); \
      } else { \
        const int jj = ii - A_INST; \
        const int dhi = jj / 9, sub = jj - dhi * 9; \
        const int row = sub * 8 + (lane >> 3); \
        const int ch = (lane & 7) ^ wg_swz<CPRX>(row); \
        const int px = unpad(u0 - 4 + row + (dhi - 1) * PW); \
        lds_dma16(xr, Xs + dhi * X_BYTES + sub * 1024, px >= 0 ? (unsigned)(((long long)px * a.ldx + c0 + ch * 8) * 2) : 0xFFFFFFF0u); \
      } \
    } \
  } while (0)

  // INC: the wave's pieces k (instruction ii = wid + 8 k): lane-constant source offsets, X rows
  constexpr int KMAX = (N_INST + 7) / 8;
  constexpr int KA = A_INST / 8;  // pieces 0 .. KA-1 of every wave are dY rows (A_INST % 8 == 0)
  static_assert(A_INST % 8 == 0, "dY pieces must be whole rounds of the 8 waves");
  unsigned loff[KMAX];
  int xrow[KMAX], xdh[KMAX];
  if constexpr (INC && !PADK) {
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int ii = wid + 8 * k;
      if (k < KA) {
        const int row = ii * RPIA + lane / CPRA;
        const int ch = (lane % CPRA) ^ wg_swz<CPRA>(row);
        loff[k] = (unsigned)(((long long)row * a.lddy + co0 + ch * 8) * 2);
        xrow[k] = 0;
        xdh[k] = 0;
      } else {
        const int jj = ii - A_INST;
        const int dhi = jj / 9, sub = jj - dhi * 9;
        const int row = sub * 8 + (lane >> 3);
        const int ch = (lane & 7) ^ wg_swz<CPRX>(row);
        loff[k] = (unsigned)(((long long)(row - 4) * a.ldx + c0 + ch * 8) * 2);
        xrow[k] = row - 4;
        xdh[k] = dhi;
      }
    }
  }
  // INC: image coordinates of the next issued K-step's first pixel (kbeg + issued * 64)
  int in_ = kbeg / HW, ipr = (kbeg - in_ * HW) / a.W, iq0 = kbeg - in_ * HW - ipr * a.W, ipx = kbeg;
  // a.band: the K-steps walk bands of a.band image rows column block by column block, so two of a
  // step's three X strips are the previous step's (L2-hot) instead of a whole row of steps back;
  // the band's first row and the row within it
  int bn_ = in_, bpr = ipr, bri = 0;
#define W9_ISSUE_INC(stage_) \
  do { \
    char* As = smem + (stage_) * STAGE; \
    char* Xs = As + A_BYTES; \
    const unsigned aso = (unsigned)((long long)(ipx - kbeg) * a.lddy * 2); \
    const long long xb = (long long)in_ * HW + (long long)ipr * a.W + iq0 - xlo; \
    _Pragma("unroll") for (int k = 0; k < KMAX; ++k) { \
      const int ii = wid + 8 * k; \
      if (k < KA) { \
        lds_dma16(dyr, As + ii * 1024, loff[k] + aso); \
      } else if (ii < N_INST) { \
        const int h = ipr + xdh[k] - 1; \
        const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)(iq0 + xrow[k]) < (unsigned)a.W; \
        const unsigned xso = (unsigned)((xb + (long long)(xdh[k] - 1) * a.W) * a.ldx * 2); \
        lds_dma16(xr, Xs + xdh[k] * X_BYTES + (ii - A_INST - xdh[k] * 9) * 1024, \
                  ok ? loff[k] + xso : 0xFFFFFFF0u); \
      } \
    } \
    if (a.band) { /* down the band's rows, then the next 64-pixel column block of the band */ \
      if (++bri == a.band) { \
        bri = 0; \
        iq0 += BKP; \
        if (iq0 == a.W) { \
          iq0 = 0; \
          bpr += a.band; \
          while (bpr >= a.H) { bpr -= a.H; ++bn_; } \
        } \
        in_ = bn_; \
        ipr = bpr; \
      } else if (++ipr == a.H) { ipr = 0; ++in_; } \
      ipx = (int)(((long long)in_ * a.H + ipr) * a.W + iq0); \
    } else { \
      ipx += BKP; \
      iq0 += BKP; \
      if (iq0 == a.W) { \
        iq0 = 0; \
        if (++ipr == a.H) { ipr = 0; ++in_; } \
      } \
    } \
  } while (0)

#define W9_ISSUE(kt_, stage_) \
  do { \
    if constexpr (PADK) { W9_ISSUE_PAD(kt_, stage_); break; } \
    if constexpr (INC) { W9_ISSUE_INC(stage_); break; } \
    const int px0 = kbeg + (kt_) * BKP; \
    const int n = px0 / HW, rem = px0 - n * HW; \
    const int pr = rem / a.W, q0 = rem - pr * a.W; \
    char* As = smem + (stage_) * STAGE; \
    char* Xs = As + A_BYTES; \
    for (int ii = wid; ii < N_INST; ii += 8) { \
      if (ii < A_INST) { \
        const int row = ii * RPIA + lane / CPRA; \
        const int ch = (lane % CPRA) ^ wg_swz<CPRA>(row); \
        lds_dma16(dyr, As + ii * 1024, (unsigned)(((long long)(px0 + row - kbeg) * a.lddy + co0 + ch * 8) * 2)); \
      } else { \
        const int jj = ii - A_INST; \
        const int dhi = jj / 9, sub = jj - dhi * 9; \
        const int row = sub * 8 + (lane >> 3); \
        const int ch = (lane & 7) ^ wg_swz<CPRX>(row); \
        const int h = pr + dhi - 1, w = q0 - 4 + row; \
        const bool ok = (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W; \
        const long long pin = (long long)n * HW + (long long)h * a.W + w - xlo; \
        lds_dma16(xr, Xs + dhi * X_BYTES + sub * 1024, ok ? (unsigned)((pin * a.ldx + c0 + ch * 8) * 2) : 0xFFFFFFF0u); \
      } \
    } \
  } while (0)

  f4v acc[9][TI][TJ];
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[tp][i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  const int wco = KH ? 0 : WIDE ? (wid & 1) * 64 : (BCO == 128 ? (wid & 3) * 32 : (wid & 1) * 32);
  const int wc = KH ? (wid & 3) * 16 : WIDE ? (wid >> 1) * 16 : (BCO == 128 ? (wid >> 2) * 32 : (wid >> 1) * 16);
  const int kh = KH ? (wid >> 2) : 0;
  const int g = lane >> 4, qq = (lane & 15) >> 2, p4 = lane & 3;
  const int hb = (p4 & 1) * 8;

  if (nkt > 0) W9_ISSUE(0, 0);
  if (nkt > 1) W9_ISSUE(1, 1);
  for (int kt = 0; kt < nkt; ++kt) {
    if (kt + 1 < nkt) {
      if (my_inst == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if (my_inst == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else if (my_inst == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (SCH == 0 && kt + 2 < nkt) W9_ISSUE(kt + 2, (kt + 2) % PSTAGES);
    const char* As = smem + (kt % PSTAGES) * STAGE;
    const char* Xs = As + A_BYTES;
#pragma unroll
    for (int ks = 0; ks < BKP / 32; ++ks) {
      if (!KH || ks == kh) {
      if constexpr (SCH == 2) __builtin_amdgcn_s_setprio(1);
      const int r1 = 32 * ks + 4 * g + qq, r2 = r1 + 16;
      s8v af[TI];
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int cc = (wco + 16 * i) / 8 + (p4 >> 1);
        s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DG_LDS s4v*)(As + r1 * RA + ((cc ^ wg_swz<CPRA>(r1)) << 4) + hb));
        s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (DG_LDS s4v*)(As + r2 * RA + ((cc ^ wg_swz<CPRA>(r2)) << 4) + hb));
        af[i] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int dhi = 0; dhi < 3; ++dhi) {
#pragma unroll
        for (int sw = 0; sw < 3; ++sw) {
          const int x1 = r1 + sw + 3, x2 = r2 + sw + 3;
          s8v bfv[TJ];
#pragma unroll
          for (int j = 0; j < TJ; ++j) {
            const int cc = (wc + 16 * j) / 8 + (p4 >> 1);
            const char* X = Xs + dhi * X_BYTES;
            s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (DG_LDS s4v*)(X + x1 * RX + ((cc ^ wg_swz<CPRX>(x1)) << 4) + hb));
            s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (DG_LDS s4v*)(X + x2 * RX + ((cc ^ wg_swz<CPRX>(x2)) << 4) + hb));
            bfv[j] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          }
#pragma unroll
          for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TJ; ++j)
              acc[dhi * 3 + sw][i][j] =
                  mfma16x16x32<T>(af[i], bfv[j], acc[dhi * 3 + sw][i][j]);
        }
      }
      if constexpr (SCH == 2) __builtin_amdgcn_s_setprio(0);
      }
      if constexpr (SCH == 2) {
        if (ks == 0 && kt + 2 < nkt) W9_ISSUE(kt + 2, (kt + 2) % PSTAGES);
      }
    }
  }
#undef W9_ISSUE
#undef W9_ISSUE_PAD
#undef W9_ISSUE_INC

  const long long ldk = 9ll * a.C;
  float* out = a.slab + ((long long)split * (KH ? 2 : 1) + kh) * a.Cout * ldk;
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        const int c = c0 + wc + 16 * j + (lane & 15);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int co = co0 + wco + 16 * i + 4 * g + rr;
          out[co * ldk + tp * a.C + c] = acc[tp][i][j][rr];
        }
      }
}

static bool wg9_inc() {  // DGVCC_WG9_INC=0: per-K-step recomputed DMA addressing (read per launch: A/B)
  const char* e = getenv("DGVCC_WG9_INC");
  return !(e && e[0] == '0');
}

static int wg9_sched() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DGVCC_WG9_SCH");
    v = (e && e[0] == '0') ? 0 : 2;
  }
  return v;
}

static bool wg9_khalf() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DGVCC_WG9_KH");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

static bool wg9_wide() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DGVCC_WG9_TILE");
    v = (e && e[0] == '0') ? 0 : 1;  // default: the 64 co x 16 c wave tile (A/B: +2% on the 128-co layers)
  }
  return v == 1;
}

static bool wg9_ok(int C, int Cout, int R, int S, int W, int pad) {
  return use_pipe() && R == 3 && S == 3 && pad == 1 && W % 64 == 0 && C % 64 == 0 && Cout % 64 == 0;
}

// the padded-K variant: any W; whole-tensor buffer descriptors (32-bit byte offsets)
static bool wg9p_ok(int N, int H, int W, int C, int Cout, int R, int S, int pad, long long ldx, long long lddy) {
  const char* e = getenv("DGVCC_WG9_PAD");
  if (e && e[0] == '0') return false;
  const long long M = (long long)N * H * W;
  return use_pipe() && R == 3 && S == 3 && pad == 1 && W % 64 != 0 && C % 64 == 0 && Cout % 64 == 0 &&
         M * std::max(ldx, lddy) * 2 < (1ll << 31) && (long long)N * (H + 2) * (W + 2) < (1ll << 30);
}


// splits for the fused-tap kernel: >= 8 K-steps per block, block count chosen for
// whole rounds of one block per CU (tail efficiency >= 90% where possible), starting from
// one round: every extra round doubles the f32 slab written and re-read by the reduce.
// units: the K index space (pixels, or padded cells for the PADK variant).
// DGVCC_WG9_BAND=0: row-major K-steps; B: bands of B rows (read per call: A/B).  Default 8 on the
// 64-input-channel layers, the HBM-bound ones (`profiles/round3d/ab_wgrad9_band*.txt`: 64 -> 64 at
// 768x1024 +5.4%, the wider layers within +-1%)
static int wg9_band(int C) {
  const char* e = getenv("DGVCC_WG9_BAND");
  return e ? std::max(0, atoi(e)) : (C == 64 ? 8 : 0);
}
// quantum: K-steps per split rounded up to a multiple of it (whole bands of rows per split)
static WgPlan wg9_plan(long long units, int C, int Cout, long long quantum = 1) {
  const long long steps = (units + 63) / 64;
  const int bco = Cout % 128 == 0 ? 128 : 64;
  const long long tiles = (long long)(Cout / bco) * (C / 64);
  long long best = 1;
  double best_eff = -1.0;
  static int rmin = -1;
  if (rmin < 0) {
    const char* e = getenv("DGVCC_WG9_ROUNDS");
    rmin = e ? std::max(1, atoi(e)) : 1;  // A/B (MI355X): 1 round beats 2 by 2% (768x1024) / 8% (320 crops)
  }
  for (int rounds = rmin; rounds <= 12; ++rounds) {
    long long sp = (256ll * rounds + tiles - 1) / tiles;
    sp = std::max(1ll, std::min(sp, std::max(1ll, steps / 8)));
    const long long blocks = tiles * sp;
    const double eff = (double)blocks / (256.0 * ((blocks + 255) / 256));
    if (eff > best_eff + 1e-9) { best_eff = eff; best = sp; }
    if (eff >= 0.9) break;
  }
  long long sps = (steps + best - 1) / best;  // K-steps per split
  if (quantum > 1) sps = (sps + quantum - 1) / quantum * quantum;
  const long long splits = (steps + sps - 1) / sps;
  return WgPlan{(int)splits, (int)(sps * 64)};
}
// the band height the 9-tap wgrad of this (W % 64 == 0) shape walks in, or 0
static int wg9_band_of(int N, int H, int W, int C) {
  const int b = wg9_band(C);
  return (b > 1 && b <= H && ((long long)N * H) % b == 0) ? b : 0;
}

// ld* < 0: the shape-only plan of the workspace query (assumes the padded 9-tap kernel is
// eligible); pad_ok = false: callers whose launch never takes the padded kernel.
template <typename T>
WgPlan wg_plan(int N, int H, int W, int C, int Cout, int R, int S, long long ldx = -1, long long lddy = -1,
               bool pad_ok = false) {  // H, W: output grid
  constexpr int BKP = WgCfg<T>::BKP;
  if (Is16<T>::value && wg9_ok(C, Cout, R, S, W, (R - 1) / 2)) {
    const int b = wg9_band_of(N, H, W, C);
    return wg9_plan((long long)N * H * W, C, Cout, b ? (long long)b * W / 64 : 1);
  }
  if (Is16<T>::value && pad_ok &&
      wg9p_ok(N, H, W, C, Cout, R, S, (R - 1) / 2, ldx < 0 ? C : ldx, lddy < 0 ? Cout : lddy))
    return wg9_plan((long long)N * (H + 2) * (W + 2), C, Cout);
  const long long M = (long long)N * H * W;
  const int bco = (Cout % 128 == 0) ? 128 : 64;
  const int bc = (C % 128 == 0) ? 128 : 64;
  const long long tiles = (long long)(Cout / bco) * (C / bc) * R * S;
  const long long max_split = (M + BKP * 4 - 1) / (BKP * 4);  // >= 4 K-tiles per block
  // Whole rounds of resident blocks (conv_wgrad_kernel: 2 per CU, 256 CUs): the blocks of a
  // split plan all run the same K length, so a grid of 2.04 rounds (the old "about 1024
  // blocks" plan: 36 tiles x 29 splits = 1044 on 512 slots) costs 3 rounds: 62% MFMA-busy
  // on the f32 layers.  Pick the fewest rounds whose last round is >= 96% full.
  const long long slots = 512;
  long long splits = 1;
  double best_eff = -1.0;
  for (int rounds = 1; rounds <= 32; ++rounds) {
    long long sp = std::max(1ll, std::min(slots * rounds / tiles, max_split));
    const long long blocks = tiles * sp;
    const double eff = (double)blocks / (double)(slots * ((blocks + slots - 1) / slots));
    if (eff > best_eff + 1e-9) { best_eff = eff; splits = sp; }
    if (eff >= 0.96 || sp == max_split) break;
  }
  if (splits < 1) splits = 1;
  long long pps = (M + splits - 1) / splits;
  pps = (pps + BKP - 1) / BKP * BKP;
  splits = (M + pps - 1) / pps;
  return WgPlan{(int)splits, (int)pps};
}

template <typename T>
int launch_wgrad(WgArgs a, float* dw, int accumulate, hipStream_t st, unsigned* hslots = nullptr) {
  const int bco = (a.Cout % 128 == 0) ? 128 : 64;
  const int bc = (a.C % 128 == 0) ? 128 : 64;
  const int tiles = (a.Cout / bco) * (a.C / bc) * a.R * a.S;
  const dim3 grid(tiles * a.splits);
  bool done = false;
  int slab_splits = a.splits;
  if constexpr (Is16<T>::value) {
    const bool w9 = a.stride == 1 && !a.whole_x && wg9_ok(a.C, a.Cout, a.R, a.S, a.W, a.pad);
    const bool w9p = a.stride == 1 && !a.whole_x && !w9 && a.pad_ok &&
                     wg9p_ok(a.N, a.H, a.W, a.C, a.Cout, a.R, a.S, a.pad, a.ldx, a.lddy);
    if (w9 || w9p) {
      const int b9 = a.Cout % 128 == 0 ? 128 : 64;
      const dim3 g9((a.Cout / b9) * (a.C / 64) * a.splits);
      const int sch = wg9_sched();
      const bool kh2 = b9 == 64 && sch == 2 && wg9_khalf();
      if (kh2) slab_splits = 2 * a.splits;  // one slab split per k-half
      if (w9) {
        const bool inc = wg9_inc();
        {
          const int b = wg9_band_of(a.N, a.H, a.W, a.C);
          a.band = (inc && b && a.pps % ((long long)b * a.W) == 0) ? b : 0;
        }
        if (b9 == 128 && wg9_wide() && sch == 2) {
          if (inc) hipLaunchKernelGGL((conv_wgrad9_kernel<128, 1, 0, 2, T>), g9, dim3(512), 0, st, a);
          else hipLaunchKernelGGL((conv_wgrad9_kernel<128, 1, 0, 2, T, 0>), g9, dim3(512), 0, st, a);
        } else if (b9 == 128 && wg9_wide()) hipLaunchKernelGGL((conv_wgrad9_kernel<128, 1, 0, 0, T, 0>), g9, dim3(512), 0, st, a);
        else if (b9 == 128) hipLaunchKernelGGL((conv_wgrad9_kernel<128, 0, 0, 0, T, 0>), g9, dim3(512), 0, st, a);
        else if (kh2) {
          if (inc) hipLaunchKernelGGL((conv_wgrad9_kernel<64, 2, 0, 2, T>), g9, dim3(512), 0, st, a);
          else hipLaunchKernelGGL((conv_wgrad9_kernel<64, 2, 0, 2, T, 0>), g9, dim3(512), 0, st, a);
        } else if (sch == 2) hipLaunchKernelGGL((conv_wgrad9_kernel<64, 0, 0, 2, T, 0>), g9, dim3(512), 0, st, a);
        else hipLaunchKernelGGL((conv_wgrad9_kernel<64, 0, 0, 0, T, 0>), g9, dim3(512), 0, st, a);
      } else {
        if (b9 == 128 && wg9_wide() && sch == 2) hipLaunchKernelGGL((conv_wgrad9_kernel<128, 1, 1, 2, T>), g9, dim3(512), 0, st, a);
        else if (b9 == 128 && wg9_wide()) hipLaunchKernelGGL((conv_wgrad9_kernel<128, 1, 1, 0, T>), g9, dim3(512), 0, st, a);
        else if (b9 == 128) hipLaunchKernelGGL((conv_wgrad9_kernel<128, 0, 1, 0, T>), g9, dim3(512), 0, st, a);
        else if (kh2) hipLaunchKernelGGL((conv_wgrad9_kernel<64, 2, 1, 2, T>), g9, dim3(512), 0, st, a);
        else if (sch == 2) hipLaunchKernelGGL((conv_wgrad9_kernel<64, 0, 1, 2, T>), g9, dim3(512), 0, st, a);
        else hipLaunchKernelGGL((conv_wgrad9_kernel<64, 0, 1, 0, T>), g9, dim3(512), 0, st, a);
      }
      done = true;
    } else if (use_wgrad_pipe()) {  // opt-in: measured slower than the register-staged kernel (round 1)
      const int RS = a.R * a.S;
      if (bco == 128 && a.C % 256 == 0) {
        hipLaunchKernelGGL((conv_wgrad_pipe_kernel<128, 256, T>), dim3((a.Cout / 128) * (a.C / 256) * RS * a.splits),
                           dim3(512), 0, st, a);
      } else if (bco == 128 && bc == 128) {
        hipLaunchKernelGGL((conv_wgrad_pipe_kernel<128, 128, T>), grid, dim3(512), 0, st, a);
      } else if (bco == 128) {
        hipLaunchKernelGGL((conv_wgrad_pipe_kernel<128, 64, T>), grid, dim3(512), 0, st, a);
      } else if (bc == 128) {
        hipLaunchKernelGGL((conv_wgrad_pipe_kernel<64, 128, T>), grid, dim3(512), 0, st, a);
      } else {
        hipLaunchKernelGGL((conv_wgrad_pipe_kernel<64, 64, T>), grid, dim3(512), 0, st, a);
      }
      done = true;
    }
  }
  if (done) {
  } else if constexpr (!Is16<T>::value) {
    const long long M3 = (long long)a.N * a.P * a.Q;
    const int b3 = wgs3_tile(a.C, a.Cout, a.R, a.S, a.W);
    const bool nr3 = wgs9_on(b3);
    if (f32_split() && a.stride == 1 && !a.whole_x && a.pad == 1 && b3) {
      const WgPlan p = nr3 ? wgs_plan(M3, wgs9_tiles(a.C, a.Cout), 256) : wgs_plan(M3, wgs3_tiles(a.C, a.Cout, b3), wgs3_slots(b3));
      if ((long long)(p.pps + 2 * (a.W + 1)) * std::max(a.ldx, a.lddy) * 4 < (1ll << 31)) {
        a.splits = p.splits;
        a.pps = p.pps;
        slab_splits = p.splits;
        const dim3 g3((unsigned)((nr3 ? wgs9_tiles(a.C, a.Cout) : wgs3_tiles(a.C, a.Cout, b3)) * p.splits));
        const bool h16 = f32_h16() && hslots;
        if (h16) {  // f16 x3: the operands' largest magnitudes (computed here unless the caller has them)
          if (!a.xam) {
            const int r = launch_camax((const float*)a.x, a.ldx, (long long)a.N * a.H * a.W, a.C, hslots, st);
            if (r != DG_OK) return r;
            a.xam = hslots;
          }
          if (!a.dyam) {
            unsigned* dys = hslots + dg_amax_words(a.C);
            const int r = launch_camax((const float*)a.dy, a.lddy, M3, a.Cout, dys, st);
            if (r != DG_OK) return r;
            a.dyam = dys;
          }
        }
        if (h16) {
          if (nr3) hipLaunchKernelGGL((conv_wgrad_split3_kernel<64, 64, 2, 512, 2, 3, 1>), g3, dim3(512), 0, st, a);
          else if (b3 == 64) hipLaunchKernelGGL((conv_wgrad_split3_kernel<64, 64, 2, 256, 0, 1, 1>), g3, dim3(256), 0, st, a);
          else hipLaunchKernelGGL((conv_wgrad_split3_kernel<128, 128, 2, 512, 2, 1, 1>), g3, dim3(512), 0, st, a);
        } else if (nr3) hipLaunchKernelGGL((conv_wgrad_split3_kernel<64, 64, 2, 512, 2, 3>), g3, dim3(512), 0, st, a);
        else if (b3 == 64) hipLaunchKernelGGL((conv_wgrad_split3_kernel<64, 64, 2, 256>), g3, dim3(256), 0, st, a);
        else {
          // placement of the next step's split + LDS stores among the taps' MFMA blocks: 0 after tap 1,
          // 1 dY after tap 0 / X after tap 1, 2 (default) all after tap 0: wgrad 0.59 -> 0.60 of the
          // ceiling (profiles/round2g/wgrad3_swp_ab.txt)
          const char* e = getenv("DGVCC_WG3_SWP");
          const int sw = e ? e[0] - '0' : 2;
          if (sw == 1) hipLaunchKernelGGL((conv_wgrad_split3_kernel<128, 128, 2, 512, 1>), g3, dim3(512), 0, st, a);
          else if (sw == 2) hipLaunchKernelGGL((conv_wgrad_split3_kernel<128, 128, 2, 512, 2>), g3, dim3(512), 0, st, a);
          else hipLaunchKernelGGL((conv_wgrad_split3_kernel<128, 128, 2, 512>), g3, dim3(512), 0, st, a);
        }
        done = true;
      }
    }
  }
  if (done) {
  } else if constexpr (!Is16<T>::value) {
    const bool wgs = f32_split() && wgs_ok(a.C, a.Cout);
    const WgPlan pw = wgs ? wgs_plan((long long)a.N * a.P * a.Q, wgs_tiles(a.C, a.Cout, a.R * a.S), wgs_slots(a.C, a.Cout))
                          : WgPlan{1, 0};
    if (wgs &&
        (long long)(pw.pps + 2 * a.pad * (a.W + 1)) * std::max(a.ldx, a.lddy) * 4 < (1ll << 31)) {
      const WgPlan p = pw;
      a.splits = p.splits;
      a.pps = p.pps;
      slab_splits = p.splits;
      const dim3 gs((unsigned)(wgs_tiles(a.C, a.Cout, a.R * a.S) * p.splits));
      const int bco = wgs_bco(a.C, a.Cout), bcw = wgs_bc(a.C, a.Cout);
      const bool h16 = f32_h16() && hslots;
      if (h16) {  // f16 x3: the operands' largest magnitudes (computed here unless the caller has them)
        if (!a.xam) {
          const int r = launch_camax((const float*)a.x, a.ldx, (long long)a.N * a.H * a.W, a.C, hslots, st);
          if (r != DG_OK) return r;
          a.xam = hslots;
        }
        if (!a.dyam) {
          unsigned* dys = hslots + dg_amax_words(a.C);
          const int r = launch_camax((const float*)a.dy, a.lddy, (long long)a.N * a.P * a.Q, a.Cout, dys, st);
          if (r != DG_OK) return r;
          a.dyam = dys;
        }
        if (bco == 64) hipLaunchKernelGGL((conv_wgrad_split_kernel<64, 64, 2, 256, 1>), gs, dim3(256), 0, st, a);
        else if (bcw == 256) hipLaunchKernelGGL((conv_wgrad_split_kernel<128, 256, 2, 512, 1>), gs, dim3(512), 0, st, a);
        else if (bcw == 128) hipLaunchKernelGGL((conv_wgrad_split_kernel<128, 128, 2, 512, 1>), gs, dim3(512), 0, st, a);
        else hipLaunchKernelGGL((conv_wgrad_split_kernel<128, 64, 4, 512, 1>), gs, dim3(512), 0, st, a);
      } else if (bco == 64) hipLaunchKernelGGL((conv_wgrad_split_kernel<64, 64, 2, 256>), gs, dim3(256), 0, st, a);
      else if (bcw == 256) hipLaunchKernelGGL((conv_wgrad_split_kernel<128, 256, 2>), gs, dim3(512), 0, st, a);
      else if (bcw == 128) hipLaunchKernelGGL((conv_wgrad_split_kernel<128, 128, 2>), gs, dim3(512), 0, st, a);
      else hipLaunchKernelGGL((conv_wgrad_split_kernel<128, 64, 4>), gs, dim3(512), 0, st, a);
      done = true;
    } else if (f32_split()) {
      if (bco == 128 && bc == 128) hipLaunchKernelGGL((conv_wgrad_kernel<T, 128, 128, 1>), grid, dim3(NT), 0, st, a);
      else if (bco == 128) hipLaunchKernelGGL((conv_wgrad_kernel<T, 128, 64, 1>), grid, dim3(NT), 0, st, a);
      else if (bc == 128) hipLaunchKernelGGL((conv_wgrad_kernel<T, 64, 128, 1>), grid, dim3(NT), 0, st, a);
      else hipLaunchKernelGGL((conv_wgrad_kernel<T, 64, 64, 1>), grid, dim3(NT), 0, st, a);
      done = true;
    }
  }
  if (done) {
  } else if (bco == 128 && bc == 128) hipLaunchKernelGGL((conv_wgrad_kernel<T, 128, 128>), grid, dim3(NT), 0, st, a);
  else if (bco == 128) hipLaunchKernelGGL((conv_wgrad_kernel<T, 128, 64>), grid, dim3(NT), 0, st, a);
  else if (bc == 128) hipLaunchKernelGGL((conv_wgrad_kernel<T, 64, 128>), grid, dim3(NT), 0, st, a);
  else hipLaunchKernelGGL((conv_wgrad_kernel<T, 64, 64>), grid, dim3(NT), 0, st, a);
  DG_CHECK_LAUNCH();
  const long long total = (long long)a.Cout * a.C * a.R * a.S;
  const int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, a.slab, slab_splits, a.Cout, a.C,
                     a.R * a.S, dw, accumulate);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// ---------------------------------------------------------------------------
// weight layout transforms
// ---------------------------------------------------------------------------
template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ w, int Cout, int C, int R, int S, int Cpad,
                                   int row_len, T* __restrict__ out) {
  const long long total = (long long)Cout * row_len;
  for (long long o = blockIdx.x * (long long)blockDim.x + threadIdx.x; o < total;
       o += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(o / row_len);
    const int k = (int)(o % row_len);
    float v = 0.f;
    if (k < R * S * Cpad) {
      const int rs = k / Cpad, c = k % Cpad;
      if (c < C) v = w[(((long long)co * C + c) * R + rs / S) * S + rs % S];
    }
    out[o] = from_f<T>(v);
  }
}

// wflip[ci][r][s][co] = w[co][R-1-r][S-1-s][ci]   (w packed [Cout][R][S][C])
template <typename T>
__global__ void flip_weight_kernel(const T* __restrict__ w, int Cout, int C, int R, int S, T* __restrict__ wf) {
  const long long total = (long long)Cout * C * R * S;
  for (long long o = blockIdx.x * (long long)blockDim.x + threadIdx.x; o < total;
       o += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(o % Cout);
    long long t = o / Cout;
    const int s = (int)(t % S); t /= S;
    const int r = (int)(t % R);
    const int ci = (int)(t / R);
    wf[o] = w[(((long long)co * R + (R - 1 - r)) * S + (S - 1 - s)) * C + ci];
  }
}

// pack_weight_kernel's default layout (Cpad = C, row_len = R*S*C) and flip_weight_kernel's wflip of the
// same stored values in one pass: a training step's per-layer filter prep in one launch instead of two
// (each ~5 us, almost all launch and ramp: 40-90 of them per step).  32-bit index math (total < 2^31,
// checked by the launcher).
template <typename T>
__global__ void pack_flip_weight_kernel(const float* __restrict__ w, int Cout, int C, int R, int S,
                                        T* __restrict__ out, T* __restrict__ wf) {
  const int RSC = R * S * C, total = Cout * RSC;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gridDim.x * blockDim.x) {
    const int co = o / RSC, k = o - co * RSC;
    const int rs = k / C, c = k - rs * C;
    const int r = rs / S, s2 = rs - r * S;
    const T v = from_f<T>(w[((co * C + c) * R + r) * S + s2]);
    out[o] = v;
    wf[((c * R + (R - 1 - r)) * S + (S - 1 - s2)) * Cout + co] = v;
  }
}

// First layer im2col: img NCHW f32 [N][3][H][W] -> out [N*H*W][64], k = (r*3+s)*3+c.
template <typename T>
__global__ void im2col_c3_kernel(const float* __restrict__ img, int N, int H, int W, T* __restrict__ out) {
  const long long M = (long long)N * H * W;
  for (long long m = blockIdx.x * (long long)blockDim.x + threadIdx.x; m < M;
       m += (long long)gridDim.x * blockDim.x) {
    const int n = (int)(m / ((long long)H * W));
    const int rem = (int)(m % ((long long)H * W));
    const int h = rem / W, w = rem % W;
    float v[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) v[k] = 0.f;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int hh = h + r - 1, ww = w + s - 1;
        if ((unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W) {
#pragma unroll
          for (int c = 0; c < 3; ++c)
            v[(r * 3 + s) * 3 + c] = img[(((long long)n * 3 + c) * H + hh) * W + ww];
        }
      }
    T* o = out + m * 64;
    constexpr int E = 16 / (int)sizeof(T);
#pragma unroll
    for (int k = 0; k < 64; k += E) stv(o + k, v + k);
  }
}

// general im2col for Cin = 3 stems: out[(n,p,q)][k], k = (r*S + s)*3 + c, zero tail to Kpad
template <typename T>
__global__ void im2col_c3_ex_kernel(const float* __restrict__ img, int N, int H, int W, int R, int S, int stride,
                                    int pad, int P, int Q, int Kpad, T* __restrict__ out) {
  // one thread per (output pixel, 16-byte chunk of k); 32-bit index math (ABI checks the sizes)
  constexpr int E = 16 / (int)sizeof(T);
  const int nch = Kpad / E, PQ = P * Q, RS3 = R * S * 3;
  const long long total = (long long)N * PQ * nch;
  for (long long o = blockIdx.x * (long long)blockDim.x + threadIdx.x; o < total;
       o += (long long)gridDim.x * blockDim.x) {
    const int m = (int)(o / nch), chk = (int)(o - (long long)m * nch);
    const int n = m / PQ, rem = m - n * PQ;
    const int p = rem / Q, q = rem - p * Q;
    const int h0 = p * stride - pad, w0 = q * stride - pad;
    const float* base = img + (long long)n * 3 * H * W;
    float v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int k = chk * E + e;
      float x = 0.f;
      if (k < RS3) {
        const int rs = k / 3, c = k - 3 * rs, r = rs / S, s2 = rs - r * S;
        const int h = h0 + r, w = w0 + s2;
        if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) x = base[((long long)c * H + h) * W + w];
      }
      v[e] = x;
    }
    stv(out + (long long)m * Kpad + chk * E, v);
  }
}

// LDS-staged form of the same im2col: a block writes I2C_QB output pixels of one output row
// (n, p, q0 ..): the 3*R input row segments they read are staged in LDS with coalesced loads
// (zeros outside the image), then each lane writes 16-byte chunks of the Kpad-wide rows from a
// per-k LDS offset table.  The one-thread-per-chunk gather above issues one scattered 4-byte
// global load (and the k -> (r, s, c) divisions) per element: 2.4 TB/s of writes (f32), 1.4 (bf16)
constexpr int I2C_QB = 64, I2C_LDS = 4096, I2C_KMAX = 256;
static bool im2col_lds_ok(int R, int S, int stride, int Kpad) {
  const char* e = getenv("DGVCC_IM2COL_LDS");  // =0: the gather kernel (A/B, read per launch)
  return !(e && e[0] == '0') && 3 * R * ((I2C_QB - 1) * stride + S) <= I2C_LDS && Kpad <= I2C_KMAX;
}
template <typename T>
__global__ __launch_bounds__(256) void im2col_c3_lds_kernel(const float* __restrict__ img, int N, int H, int W, int R,
                                                            int S, int stride, int pad, int P, int Q, int Kpad,
                                                            T* __restrict__ out) {
  __shared__ float seg[I2C_LDS];
  __shared__ int koff[I2C_KMAX];
  constexpr int E = 16 / (int)sizeof(T);
  const int tid = threadIdx.x, qb = (Q + I2C_QB - 1) / I2C_QB;
  const int b = blockIdx.x, n = b / (P * qb), rem = b - n * P * qb, p = rem / qb, q0 = (rem - p * qb) * I2C_QB;
  const int Wl = (I2C_QB - 1) * stride + S, RS3 = R * S * 3;
  const int h0 = p * stride - pad, w0 = q0 * stride - pad;
  const float* base = img + (long long)n * 3 * H * W;
  for (int i = tid; i < 3 * R * Wl; i += 256) {
    const int row = i / Wl, j = i - row * Wl, c = row / R, r = row - c * R;
    const int h = h0 + r, w = w0 + j;
    seg[i] = ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) ? base[((long long)c * H + h) * W + w] : 0.f;
  }
  for (int k = tid; k < Kpad; k += 256) {
    int o = -1;
    if (k < RS3) {
      const int rs = k / 3, c = k - 3 * rs, r = rs / S, s2 = rs - r * S;
      o = (c * R + r) * Wl + s2;
    }
    koff[k] = o;
  }
  __syncthreads();
  const int nq = min(I2C_QB, Q - q0), nch = Kpad / E;
  T* orow = out + ((long long)(n * P + p) * Q + q0) * Kpad;
  for (int i = tid; i < nq * nch; i += 256) {
    const int qi = i / nch, chk = i - qi * nch;
    float v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int o = koff[chk * E + e];
      v[e] = o >= 0 ? seg[o + qi * stride] : 0.f;
    }
    stv(orow + (long long)qi * Kpad + chk * E, v);
  }
}

__global__ void unpack_c3_ex_kernel(const float* __restrict__ dwcol, int Cout, int R, int S, int Kpad,
                                    float* __restrict__ dw, int acc) {
  const int total = Cout * 3 * R * S;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gridDim.x * blockDim.x) {
    const int co = o / (3 * R * S), k = o % (3 * R * S);  // torch layout k = (c*R + r)*S + s
    const int c = k / (R * S), r = (k / S) % R, s = k % S;
    const float v = dwcol[(long long)co * Kpad + (r * S + s) * 3 + c];
    dw[o] = acc ? dw[o] + v : v;
  }
}

__global__ void unpack_c3_grad_kernel(const float* __restrict__ dwcol, int Cout, float* __restrict__ dw, int acc) {
  const int total = Cout * 27;
  for (int o = blockIdx.x * blockDim.x + threadIdx.x; o < total; o += gridDim.x * blockDim.x) {
    const int co = o / 27, k = o % 27;  // torch layout k = c*9 + r*3 + s
    const int c = k / 9, r = (k / 3) % 3, s = k % 3;
    const float v = dwcol[co * 64 + (r * 3 + s) * 3 + c];
    dw[o] = acc ? dw[o] + v : v;
  }
}

inline int grid_for(long long n, int bs = 256, int cap = 65536) {
  long long g = (n + bs - 1) / bs;
  if (g < 1) g = 1;
  return (int)std::min<long long>(g, cap);
}

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" int dg_version(void) { return DGVCC_ABI_VERSION; }

// Test hook: force the persistent pipelined forward on (1) / off (0), or back to the
// DGVCC_PERSIST environment default (-1).
extern "C" int dg_set_f32_math(int mode) {
  DG_REQUIRE(mode >= 0 && mode <= 2);
  g_f32_math = mode;
  return DG_OK;
}

extern "C" int dg_get_f32_math(void) { return f32_math(); }

extern "C" int dg_amax(int dtype, const void* x, int64_t ldx, int64_t M, int C, float* out, void* stream) {
  DG_REQUIRE(x && out && M >= 0 && C > 0 && ldx >= C);
  DG_SUPPORTED(dtype == DG_F32 && C % 4 == 0 && ldx % 4 == 0 && C <= DG_CAMAX_C);
  return launch_camax((const float*)x, ldx, M, C, (unsigned*)out, (hipStream_t)stream);
}

extern "C" int dg_debug_stamps(void* buf, int64_t bytes) {
  DG_REQUIRE(bytes >= 0 && (buf || bytes == 0));
  g_stamps = (unsigned long long*)buf;
  g_stamp_bytes = bytes;
  return DG_OK;
}

extern "C" int dg_set_persist(int mode) {
  DG_REQUIRE(mode >= -1 && mode <= 1);
  g_persist_override = mode;
  return DG_OK;
}

extern "C" int dg_conv_fwd(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, const void* w,
                           int Cout, int R, int S, int pad, const float* bias, void* y, int64_t ldy,
                           int accumulate, void* stream) {
  DG_REQUIRE(x && w && y && N > 0 && H > 0 && W > 0 && C > 0 && Cout > 0 && R > 0 && S > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(2 * pad == R - 1 && 2 * pad == S - 1);
  DG_SUPPORTED(Cout % 64 == 0);
  DG_SUPPORTED(DG_IS16(dtype) ? (C % 64 == 0) : (C % 32 == 0));
  DG_REQUIRE(ldx >= C && ldy >= Cout && ldx % 8 == 0 && ldy % 4 == 0);
  DG_SUPPORTED((long long)(128 + 2 * pad * (W + 1)) * ldx * 4 < (1ll << 31));
  FwdArgs a{(const char*)x, ldx, N, H, W, C, (const char*)w, Cout, R, S, pad, bias, (char*)y, ldy, accumulate};
  hipStream_t st = (hipStream_t)stream;
  return dtype == DG_BF16 ? launch_fwd<bf16>(a, st) : dtype == DG_F16 ? launch_fwd<f16>(a, st) : launch_fwd<float>(a, st);
}

// Which forward kernel serves this shape (bf16): 1 = pipelined / fused 3-tap (epilogue
// statistics available), 0 = register-staged.
static bool fwd_has_epi_stats(int C, int Cout, long long ldx, int R, int S) {
  return use_pipe() && C % 64 == 0 && ldx % 8 == 0 && (long long)Cout * R * S * C * 2 < (1ll << 31);
}

extern "C" int64_t dg_conv_stats_rows(int N, int H, int W) {
  if (N <= 0 || H <= 0 || W <= 0) return DG_ERR_INVALID;
  return dg_cdiv((long long)N * H * W, 256);
}

// rows of BN statistics partials a dg_conv_fwd_ex launch of this shape writes (one per tile
// of 256 pixels, 192 on the pre-split f32 kernel)
extern "C" int64_t dg_conv_stats_rows_ex(int dtype, int N, int H, int W, int C, int64_t ldx, int Cout, int R, int S) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || Cout <= 0 || R <= 0 || S <= 0) return DG_ERR_INVALID;
  const long long M = (long long)N * H * W;
  FwdArgs a{nullptr, ldx, N, H, W, C, nullptr, Cout, R, S, (R - 1) / 2, nullptr, nullptr, Cout, 0};
  if (dtype == DG_F32 && psplit_ok(a)) return dg_cdiv(M, psplit_tile_px(a));
  if (dtype == DG_F32 && rsplit_ok(a) && rsplit3w_ok(a)) return dg_cdiv(M, 512);
  if (DG_IS16(dtype) && pers16_wide(a)) return dg_cdiv(M, 384);
  return dg_cdiv(M, 256);
}
extern "C" int64_t dg_conv_bnpart_rows_ex(int dtype, int N, int H, int W, int C, int64_t ldx, int Cout, int R, int S) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || Cout <= 0 || R <= 0 || S <= 0) return DG_ERR_INVALID;
  const long long M = (long long)N * H * W;
  FwdArgs a{nullptr, ldx, N, H, W, C, nullptr, Cout, R, S, (R - 1) / 2, nullptr, nullptr, Cout, 0};
  if (dtype == DG_F32 && psplit_ok(a)) return dg_cdiv(M, psplit_psb(f32_pers_bn(Cout), psplit_wide()));
  return dg_cdiv(M, 256);
}
extern "C" int dg_conv_fwd_stats(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, const void* w,
                                 int Cout, int R, int S, int pad, const float* bias, void* y, int64_t ldy, float* part,
                                 void* stream) {
  DG_REQUIRE(x && w && y && part && N > 0 && H > 0 && W > 0 && C > 0 && Cout > 0 && R > 0 && S > 0);
  DG_SUPPORTED(DG_IS16(dtype) && fwd_has_epi_stats(C, Cout, ldx, R, S));
  DG_SUPPORTED(2 * pad == R - 1 && 2 * pad == S - 1 && Cout % 64 == 0);
  DG_REQUIRE(ldx >= C && ldy >= Cout && ldy % 4 == 0);
  DG_SUPPORTED((long long)(128 + 2 * pad * (W + 1)) * ldx * 4 < (1ll << 31));
  FwdArgs a{(const char*)x, ldx, N, H, W, C, (const char*)w, Cout, R, S, pad, bias, (char*)y, ldy, 0, part};
  {
    FwdArgs q = a;
    q.part = nullptr;
    if (Cout == 64 && R == 3 && S == 3 && pad == 1 && tap3_pad_ok(q)) return DG_ERR_UNSUPPORTED;
  }
  return dtype == DG_F16 ? launch_fwd<f16>(a, (hipStream_t)stream) : launch_fwd<bf16>(a, (hipStream_t)stream);
}

extern "C" int64_t dg_conv_fwd_workspace(int dtype, int N, int H, int W, int C, int Cout, int R, int S) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || Cout <= 0 || R <= 0 || S <= 0) return DG_ERR_INVALID;
  const long long M = (long long)N * H * W;
  if (dtype == DG_F32) {  // pre-split filter planes (+ the pre-split pixel operand of the f16 x3 pre-split forward)
    const long long planes = ((long long)Cout * R * S * C * 6 + 255) / 256 * 256;
    FwdArgs a{nullptr, C, N, H, W, C, nullptr, Cout, R, S, (R - 1) / 2, nullptr, nullptr, Cout, 0, nullptr};
    // room only where the launch takes the pre-split operand (psplit_xs with the shape's tile: several
    // output-channel tiles share a pixel tile of a 3x3 conv; DGVCC_PSPLIT_XS is read here too): a
    // launch given less room splits in-kernel (bit-identical), so a cached size stays safe
    if (2 * a.pad == R - 1 && 2 * a.pad == S - 1 && psplit_ok(a) && psplit_xs(a, f32_pers_bn(Cout)))
      return xsplit_off(planes) + xsplit_bytes(a);
    return planes;
  }
  if (!DG_IS16(dtype) || !fwd_has_epi_stats(C, Cout, C, R, S)) return 0;
  const int ks = fwd_ksplit(M, Cout, C, R, S);
  return ks > 1 ? (int64_t)ks * M * Cout * 4 : 0;
}

// dg_conv_fwd / dg_conv_fwd_stats with a workspace: part may be NULL (no statistics);
// a workspace of dg_conv_fwd_workspace bytes lets a small-grid shape split its K loop.
static int conv_fwd_ex_impl(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, const void* w, int Cout,
                            int R, int S, int pad, const float* bias, void* y, int64_t ldy, int accumulate,
                            float* part, void* workspace, int64_t ws_bytes, const float* xamax, const void* xpair,
                            const float* xbound, void* stream) {
  DG_REQUIRE(x && w && y && N > 0 && H > 0 && W > 0 && C > 0 && Cout > 0 && R > 0 && S > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(2 * pad == R - 1 && 2 * pad == S - 1 && Cout % 64 == 0);
  DG_SUPPORTED(DG_IS16(dtype) ? (C % 64 == 0) : (C % 32 == 0));
  DG_REQUIRE(ldx >= C && ldy >= Cout && ldx % 8 == 0 && ldy % 4 == 0);
  DG_SUPPORTED((long long)(128 + 2 * pad * (W + 1)) * ldx * 4 < (1ll << 31));
  FwdArgs a{(const char*)x, ldx, N, H, W, C, (const char*)w, Cout, R, S, pad, bias, (char*)y, ldy, accumulate, part};
  if (dtype == DG_F32) {
    a.wsplit = (char*)workspace;
    a.wsplit_bytes = workspace ? ws_bytes : 0;
    a.xamax = xamax;
    a.xpair = (const char*)xpair;
    a.xbound = xbound;
  }
  if (part) {
    if (DG_IS16(dtype)) {
      DG_SUPPORTED(fwd_has_epi_stats(C, Cout, ldx, R, S));
    } else if (psplit_ok(a) || (rsplit_ok(a) && rsplit3w_ok(a))) {
      // dg_conv_stats_rows_ex reports the pre-split kernels' rows (192/256/384- or 512-pixel tiles):
      // without room for the planes the launch would fall back to the 256-pixel persistent kernel
      // and write another row count than the caller allocated
      DG_SUPPORTED(has_split_room(a));
    } else {
      DG_SUPPORTED(f32_pers_ok(a) || (rsplit_ok(a) && has_split_room(a)));
    }
  }
  {  // the padded 3-tap kernel (faster, no epilogue statistics) serves this shape: the caller
     // runs dg_conv_fwd + the statistics pass instead
    FwdArgs q = a;
    q.part = nullptr;
    if (part && DG_IS16(dtype) && Cout == 64 && R == 3 && S == 3 && pad == 1 && tap3_pad_ok(q))
      return DG_ERR_UNSUPPORTED;
  }
  if (DG_IS16(dtype) && workspace && fwd_has_epi_stats(C, Cout, ldx, R, S)) {
    const long long M = (long long)N * H * W;
    const int ks = fwd_ksplit(M, Cout, C, R, S);
    if (ks > 1 && ws_bytes >= (int64_t)ks * M * Cout * 4) {
      a.ksplit = ks;
      a.kpart = (float*)workspace;
    }
  }
  hipStream_t st = (hipStream_t)stream;
  return dtype == DG_BF16 ? launch_fwd<bf16>(a, st) : dtype == DG_F16 ? launch_fwd<f16>(a, st) : launch_fwd<float>(a, st);
}

extern "C" int dg_conv_fwd_ex(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, const void* w,
                              int Cout, int R, int S, int pad, const float* bias, void* y, int64_t ldy,
                              int accumulate, float* part, void* workspace, int64_t ws_bytes, const float* xamax,
                              void* stream) {
  return conv_fwd_ex_impl(dtype, x, ldx, N, H, W, C, w, Cout, R, S, pad, bias, y, ldy, accumulate, part, workspace,
                          ws_bytes, xamax, nullptr, nullptr, stream);
}

// dg_conv_fwd_ex whose f32 input also comes as its producer's f16 x3 pair image (include/dgvcc.h)
extern "C" int dg_conv_fwd_pair(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, const void* w,
                                int Cout, int R, int S, int pad, const float* bias, void* y, int64_t ldy,
                                int accumulate, float* part, void* workspace, int64_t ws_bytes, const float* xamax,
                                const void* xpair, const float* xbound, void* stream) {
  DG_REQUIRE(dtype == DG_F32 && (xpair == nullptr) == (xbound == nullptr));
  DG_REQUIRE(!xpair || C % 32 == 0);
  return conv_fwd_ex_impl(dtype, x, ldx, N, H, W, C, w, Cout, R, S, pad, bias, y, ldy, accumulate, part, workspace,
                          ws_bytes, xamax, xpair, xbound, stream);
}

// y = (relu_out > 0) ? conv(x, w) + y : 0 -- the accumulating dgrad of a 1x1 conv whose input is
// the ReLU output relu_out (a bottleneck's conv1 on the previous block's output), with that ReLU's
// backward folded into the epilogue (dg_conv_fwd_ex with accumulate = 1 followed by dg_relu_bwd
// on y, bit for bit, without the extra pass over y).  w: the flipped filter (dg_flip_weight).
// DG_ERR_UNSUPPORTED (nothing launched) for the split-K shapes dg_conv_fwd_ex would split with
// this workspace: the caller runs the two launches.
extern "C" int dg_conv_fwd_acc_relu(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C,
                                    const void* w, int Cout, const void* relu_out, int64_t ldr, void* y,
                                    int64_t ldy, void* workspace, int64_t ws_bytes, const float* xamax,
                                    void* stream) {
  DG_REQUIRE(x && w && y && relu_out && N > 0 && H > 0 && W > 0 && C > 0 && Cout > 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(Cout % 64 == 0 && (DG_IS16(dtype) ? (C % 64 == 0) : (C % 32 == 0)));
  DG_REQUIRE(ldx >= C && ldy >= Cout && ldr >= Cout && ldx % 8 == 0 && ldy % 4 == 0 && ldr % 4 == 0);
  DG_SUPPORTED((long long)128 * ldx * 4 < (1ll << 31));
  FwdArgs a{(const char*)x, ldx, N, H, W, C, (const char*)w, Cout, 1, 1, 0, nullptr, (char*)y, ldy, 1, nullptr};
  a.rmask = (const char*)relu_out;
  a.ldrm = ldr;
  if (dtype == DG_F32) {
    a.wsplit = (char*)workspace;
    a.wsplit_bytes = workspace ? ws_bytes : 0;
    a.xamax = xamax;
  }
  if (DG_IS16(dtype) && workspace && fwd_has_epi_stats(C, Cout, ldx, 1, 1)) {
    const long long M = (long long)N * H * W;
    const int ks = fwd_ksplit(M, Cout, C, 1, 1);
    if (ks > 1 && ws_bytes >= (int64_t)ks * M * Cout * 4) return DG_ERR_UNSUPPORTED;
  }
  hipStream_t st = (hipStream_t)stream;
  return dtype == DG_BF16 ? launch_fwd<bf16>(a, st) : dtype == DG_F16 ? launch_fwd<f16>(a, st) : launch_fwd<float>(a, st);
}

// dgrad (or any bf16 pipelined forward) that also emits the BatchNorm-backward partial sums
// of the layer whose output gradient y is: bpart[dg_conv_stats_rows][3][Cout] for
// dg_bn_bwd_from_part.  z/ldz, scale/shift/mean/invstd, act, drop, HW describe that layer
// (dg_bn_bwd's arguments).  DG_ERR_UNSUPPORTED (nothing launched) where the shape is not
// served by the pipelined kernel in one pass (no split-K here): the caller then runs
// dg_conv_fwd + dg_bn_bwd.
// Eval-mode Conv + BatchNorm(running statistics) [+ ReLU] in one pass: the BN scale/shift
// (gamma/sqrt(running_var+eps), beta - running_mean*scale) and the activation are applied in the conv
// epilogue, so z is never written and re-read.  The f32 result equals dg_conv_fwd followed
// by dg_bn_apply bit for bit (same fmaf on the same f32 value); bf16 skips z's rounding.
extern "C" int dg_conv_fwd_bn_eval(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, const void* w,
                                   int Cout, int R, int S, int pad, const float* bias, const float* scale,
                                   const float* shift, int act, void* y, int64_t ldy, void* workspace,
                                   int64_t ws_bytes, const float* xamax, void* stream) {
  DG_REQUIRE(x && w && y && scale && shift && N > 0 && H > 0 && W > 0 && C > 0 && Cout > 0 && R > 0 && S > 0 &&
             (act == 0 || act == 1));
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(2 * pad == R - 1 && 2 * pad == S - 1 && Cout % 64 == 0);
  DG_SUPPORTED(DG_IS16(dtype) ? (C % 64 == 0) : (C % 32 == 0));
  DG_REQUIRE(ldx >= C && ldy >= Cout && ldx % 8 == 0 && ldy % 4 == 0);
  DG_SUPPORTED((long long)(128 + 2 * pad * (W + 1)) * ldx * 4 < (1ll << 31));
  FwdArgs a{(const char*)x, ldx, N, H, W, C, (const char*)w, Cout, R, S, pad, bias, (char*)y, ldy, 0};
  a.escale = scale;
  a.eshift = shift;
  a.eact = act;
  if (dtype == DG_F32) {
    a.wsplit = (char*)workspace;
    a.wsplit_bytes = workspace ? ws_bytes : 0;
    a.xamax = xamax;
  }
  if (DG_IS16(dtype) && workspace && fwd_has_epi_stats(C, Cout, ldx, R, S)) {
    const long long M = (long long)N * H * W;
    const int ks = fwd_ksplit(M, Cout, C, R, S);
    if (ks > 1 && ws_bytes >= (int64_t)ks * M * Cout * 4) {
      a.ksplit = ks;
      a.kpart = (float*)workspace;
    }
  }
  hipStream_t st = (hipStream_t)stream;
  return dtype == DG_BF16 ? launch_fwd<bf16>(a, st) : dtype == DG_F16 ? launch_fwd<f16>(a, st) : launch_fwd<float>(a, st);
}

extern "C" int dg_conv_fwd_bnbwd(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, const void* w,
                                 int Cout, int R, int S, int pad, void* y, int64_t ldy, const void* z, int64_t ldz,
                                 const float* scale, const float* shift, const float* mean, const float* invstd,
                                 int act, const float* drop, int HW, float* bpart, void* workspace, int64_t ws_bytes,
                                 const float* xamax, void* stream) {
  DG_REQUIRE(x && w && y && z && bpart && scale && shift && mean && invstd && N > 0 && H > 0 && W > 0 && C > 0 &&
             Cout > 0 && R > 0 && S > 0 && (act == 0 || act == 1) && (!drop || HW > 0));
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(dtype == DG_F32 || fwd_has_epi_stats(C, Cout, ldx, R, S));
  DG_SUPPORTED(2 * pad == R - 1 && 2 * pad == S - 1 && Cout % 128 == 0);  // the pipe kernel's 128/256 tiles
  DG_REQUIRE(ldx >= C && ldy >= Cout && ldy % 4 == 0 && ldz >= Cout && ldz % 4 == 0);
  DG_SUPPORTED((long long)(128 + 2 * pad * (W + 1)) * ldx * 4 < (1ll << 31));
  const long long M = (long long)N * H * W;
  DG_SUPPORTED(dtype == DG_F32 || fwd_ksplit(M, Cout, C, R, S) == 1);
  FwdArgs a{(const char*)x, ldx, N, H, W, C, (const char*)w, Cout, R, S, pad, nullptr, (char*)y, ldy, 0};
  a.bz = (const char*)z;
  a.ldbz = ldz;
  a.bsc = scale; a.bsf = shift; a.bmu = mean; a.bis = invstd; a.bdrop = drop;
  a.bact = act; a.bHW = drop ? HW : 1;
  a.bpart = bpart;
  if (dtype == DG_F32) {  // conv_fwd_psplit_kernel<.., EPI 2> on the caller's pre-split planes
    a.wsplit = (char*)workspace;
    a.wsplit_bytes = workspace ? ws_bytes : 0;
    a.xamax = xamax;
    return launch_fwd<float>(a, (hipStream_t)stream);
  }
  return dtype == DG_F16 ? launch_fwd<f16>(a, (hipStream_t)stream) : launch_fwd<bf16>(a, (hipStream_t)stream);
}

extern "C" int dg_flip_weight(int dtype, const void* w, int Cout, int C, int R, int S, void* wflip, void* stream) {
  DG_REQUIRE(w && wflip && Cout > 0 && C > 0 && R > 0 && S > 0);
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)Cout * C * R * S;
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(flip_weight_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, st, (const bf16*)w, Cout, C, R,
                       S, (bf16*)wflip);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(flip_weight_kernel<f16>, dim3(grid_for(total)), dim3(256), 0, st, (const f16*)w, Cout, C, R,
                       S, (f16*)wflip);
  else if (dtype == DG_F32)
    hipLaunchKernelGGL(flip_weight_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)w, Cout, C,
                       R, S, (float*)wflip);
  else
    return DG_ERR_INVALID;
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_conv_dgrad(int dtype, const void* dy, int64_t lddy, int N, int H, int W, int Cout, const void* w,
                             int C, int R, int S, int pad, void* wflip, void* dx, int64_t lddx, int accumulate,
                             void* stream) {
  DG_REQUIRE(dy && w && wflip && dx);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(C % 64 == 0);
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)Cout * C * R * S;
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(flip_weight_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, st, (const bf16*)w, Cout, C, R,
                       S, (bf16*)wflip);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(flip_weight_kernel<f16>, dim3(grid_for(total)), dim3(256), 0, st, (const f16*)w, Cout, C, R,
                       S, (f16*)wflip);
  else
    hipLaunchKernelGGL(flip_weight_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)w, Cout, C,
                       R, S, (float*)wflip);
  DG_CHECK_LAUNCH();
  return dg_conv_fwd(dtype, dy, lddy, N, H, W, Cout, wflip, C, R, S, R - 1 - pad, nullptr, dx, lddx, accumulate,
                     stream);
}

static int64_t wg_amax_bytes(int C, int Cout) {
  return (int64_t)(dg_amax_words(C) + dg_amax_words(Cout)) * 4 / 256 * 256 + 256;
}

extern "C" int64_t dg_conv_wgrad_workspace(int dtype, int N, int H, int W, int C, int Cout, int R, int S) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || Cout <= 0 || R <= 0 || S <= 0) return DG_ERR_INVALID;
  WgPlan p = DG_IS16(dtype) ? wg_plan<bf16>(N, H, W, C, Cout, R, S, -1, -1, true)
                              : wg_plan<float>(N, H, W, C, Cout, R, S);
  // the padded 9-tap plan may be refused at launch (pixel strides too large): cover the
  // fallback plan too
  WgPlan q = DG_IS16(dtype) ? wg_plan<bf16>(N, H, W, C, Cout, R, S) : p;
  if (!DG_IS16(dtype) && wgs_ok(C, Cout))
    q = wgs_plan((long long)N * H * W, wgs_tiles(C, Cout, R * S), wgs_slots(C, Cout));
  if (!DG_IS16(dtype) && wgs3_shape_ok(C, Cout, R, S, W)) {  // the 3-tap plan (launch may refuse it)
    const int b3 = wgs3_tile(C, Cout, R, S, W);
    const WgPlan q3 = wgs_plan((long long)N * H * W, wgs3_tiles(C, Cout, b3), wgs3_slots(b3));
    if (q3.splits > q.splits) q = q3;
    const WgPlan q9 = wgs_plan((long long)N * H * W, wgs9_tiles(C, Cout), 256);
    if (wgs9_on(b3) && q9.splits > q.splits) q = q9;
  }
  const int kh = (DG_IS16(dtype) && Cout % 128 != 0) ? 2 : 1;  // 9-tap Cout-64 kernel: a slab split per k-half
  // f32: + the f16 x3 operand maxima the library computes when the caller has none (dg_conv_wgrad):
  // [1 + C] for x, [1 + Cout] for dy, at the end
  return (int64_t)std::max(p.splits, q.splits) * kh * Cout * C * R * S * 4 + (DG_IS16(dtype) ? 0 : wg_amax_bytes(C, Cout));
}

extern "C" int dg_conv_wgrad(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, const void* dy,
                             int64_t lddy, int Cout, int R, int S, int pad, float* dw, void* workspace,
                             int64_t ws_bytes, int accumulate, const float* xamax, const float* dyamax,
                             void* stream) {
  DG_REQUIRE(x && dy && dw && workspace);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(2 * pad == R - 1 && 2 * pad == S - 1);
  DG_SUPPORTED(Cout % 64 == 0 && C % 64 == 0);
  DG_REQUIRE(ldx % 8 == 0 && lddy % 8 == 0 && ldx >= C && lddy >= Cout);
  const int64_t need = dg_conv_wgrad_workspace(dtype, N, H, W, C, Cout, R, S);
  DG_REQUIRE(ws_bytes >= need);
  WgPlan p = DG_IS16(dtype) ? wg_plan<bf16>(N, H, W, C, Cout, R, S, ldx, lddy, true)
                              : wg_plan<float>(N, H, W, C, Cout, R, S);
  const bool padk = DG_IS16(dtype) && !wg9_ok(C, Cout, R, S, W, pad) &&
                    wg9p_ok(N, H, W, C, Cout, R, S, pad, ldx, lddy);
  if (!padk) DG_SUPPORTED((long long)(p.pps + 2 * pad * (W + 1)) * std::max(ldx, lddy) * 4 < (1ll << 31));
  WgArgs a{(const char*)x, ldx, N, H, W, C, (const char*)dy, lddy, Cout, R, S, pad, (float*)workspace, p.splits, p.pps,
           1, H, W, 0};
  a.pad_ok = 1;
  a.xam = (const unsigned*)xamax;
  a.dyam = (const unsigned*)dyamax;
  hipStream_t st = (hipStream_t)stream;
  unsigned* hslots = dtype == DG_F32 ? (unsigned*)((char*)workspace + need - wg_amax_bytes(C, Cout)) : nullptr;
  return dtype == DG_BF16 ? launch_wgrad<bf16>(a, dw, accumulate, st) : dtype == DG_F16 ? launch_wgrad<f16>(a, dw, accumulate, st) : launch_wgrad<float>(a, dw, accumulate, st, hslots);
}

extern "C" int dg_pack_weight(int dtype, const float* w, int Cout, int C, int R, int S, int Cpad, int row_len,
                              void* out, void* stream) {
  DG_REQUIRE(w && out && Cout > 0 && C > 0 && Cpad >= C && row_len >= R * S * Cpad);
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)Cout * row_len;
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(pack_weight_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, st, w, Cout, C, R, S, Cpad,
                       row_len, (bf16*)out);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(pack_weight_kernel<f16>, dim3(grid_for(total)), dim3(256), 0, st, w, Cout, C, R, S, Cpad,
                       row_len, (f16*)out);
  else if (dtype == DG_F32)
    hipLaunchKernelGGL(pack_weight_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, w, Cout, C, R, S, Cpad,
                       row_len, (float*)out);
  else
    return DG_ERR_INVALID;
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_pack_weight_flip(int dtype, const float* w, int Cout, int C, int R, int S, void* out, void* wflip,
                                   void* stream) {
  DG_REQUIRE(w && out && wflip && Cout > 0 && C > 0 && R > 0 && S > 0);
  DG_SUPPORTED((long long)Cout * C * R * S < (1LL << 31));
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)Cout * C * R * S;
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(pack_flip_weight_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, st, w, Cout, C, R, S,
                       (bf16*)out, (bf16*)wflip);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(pack_flip_weight_kernel<f16>, dim3(grid_for(total)), dim3(256), 0, st, w, Cout, C, R, S,
                       (f16*)out, (f16*)wflip);
  else if (dtype == DG_F32)
    hipLaunchKernelGGL(pack_flip_weight_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, w, Cout, C, R, S,
                       (float*)out, (float*)wflip);
  else
    return DG_ERR_INVALID;
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_im2col3x3_c3(int dtype, const float* img, int N, int H, int W, void* out, void* stream) {
  DG_REQUIRE(img && out && N > 0 && H > 0 && W > 0);
  hipStream_t st = (hipStream_t)stream;
  const long long M = (long long)N * H * W;
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(im2col_c3_kernel<bf16>, dim3(grid_for(M, 256, 1 << 20)), dim3(256), 0, st, img, N, H, W,
                       (bf16*)out);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(im2col_c3_kernel<f16>, dim3(grid_for(M, 256, 1 << 20)), dim3(256), 0, st, img, N, H, W,
                       (f16*)out);
  else if (dtype == DG_F32)
    hipLaunchKernelGGL(im2col_c3_kernel<float>, dim3(grid_for(M, 256, 1 << 20)), dim3(256), 0, st, img, N, H, W,
                       (float*)out);
  else
    return DG_ERR_INVALID;
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_unpack_c3_grad(const float* dwcol, int Cout, float* dw, int accumulate, void* stream) {
  DG_REQUIRE(dwcol && dw && Cout > 0);
  hipLaunchKernelGGL(unpack_c3_grad_kernel, dim3(grid_for(Cout * 27)), dim3(256), 0, (hipStream_t)stream, dwcol,
                     Cout, dw, accumulate);
  DG_CHECK_LAUNCH();
  return DG_OK;
}


// ---------------------------------------------------------------------------
// general (strided) convolution C-ABI
// ---------------------------------------------------------------------------
static inline int conv_out(int in, int R, int stride, int pad) { return (in + 2 * pad - R) / stride + 1; }

extern "C" int dg_conv2d_fwd(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, const void* w,
                             int Cout, int R, int S, int stride, int pad, const float* bias, void* y, int64_t ldy,
                             int accumulate, void* stream) {
  DG_REQUIRE(x && w && y && N > 0 && H > 0 && W > 0 && C > 0 && Cout > 0 && R > 0 && S > 0 && stride >= 1 && pad >= 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(Cout % 64 == 0 && (DG_IS16(dtype) ? (C % 64 == 0) : (C % 32 == 0)));
  DG_REQUIRE(ldx >= C && ldy >= Cout && ldx % 8 == 0 && ldy % 4 == 0);
  DG_SUPPORTED((((long long)N * H * W - 1) * ldx + C) * (DG_IS16(dtype) ? 2 : 4) < (1ll << 31));
  const int P = conv_out(H, R, stride, pad), Q = conv_out(W, S, stride, pad);
  DG_REQUIRE(P > 0 && Q > 0);
  GenArgs a{(const char*)x, ldx, N, H, W, C, P, Q, (const char*)w, Cout, R, S, stride, pad, 0, bias, (char*)y, ldy,
            accumulate};
  hipStream_t st = (hipStream_t)stream;
  return dtype == DG_BF16 ? launch_gen<bf16>(a, st) : dtype == DG_F16 ? launch_gen<f16>(a, st) : launch_gen<float>(a, st);
}

extern "C" int dg_transpose_weight(int dtype, const void* w, int Cout, int C, int R, int S, void* wt, void* stream) {
  DG_REQUIRE(w && wt && Cout > 0 && C > 0 && R > 0 && S > 0);
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)Cout * C * R * S;
  if (dtype == DG_BF16)
    hipLaunchKernelGGL(transpose_weight_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, st, (const bf16*)w, Cout, C,
                       R, S, (bf16*)wt);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(transpose_weight_kernel<f16>, dim3(grid_for(total)), dim3(256), 0, st, (const f16*)w, Cout, C,
                       R, S, (f16*)wt);
  else if (dtype == DG_F32)
    hipLaunchKernelGGL(transpose_weight_kernel<float>, dim3(grid_for(total)), dim3(256), 0, st, (const float*)w, Cout,
                       C, R, S, (float*)wt);
  else
    return DG_ERR_INVALID;
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// dX [N,H,W,C] of a conv x[N,H,W,C] -> y[N,P,Q,Cout]: transposed gather of dY with
// wt = dg_transpose_weight(w) ([C][R][S][Cout]).
extern "C" int dg_conv2d_dgrad(int dtype, const void* dy, int64_t lddy, int N, int P, int Q, int Cout, const void* wt,
                               int C, int H, int W, int R, int S, int stride, int pad, void* dx, int64_t lddx,
                               int accumulate, void* stream) {
  DG_REQUIRE(dy && wt && dx && N > 0 && P > 0 && Q > 0 && H > 0 && W > 0 && stride >= 1 && pad >= 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(C % 64 == 0 && (DG_IS16(dtype) ? (Cout % 64 == 0) : (Cout % 32 == 0)));
  DG_REQUIRE(conv_out(H, R, stride, pad) == P && conv_out(W, S, stride, pad) == Q);
  DG_REQUIRE(lddy % 8 == 0 && lddx % 4 == 0);
  DG_SUPPORTED((((long long)N * P * Q - 1) * lddy + Cout) * (DG_IS16(dtype) ? 2 : 4) < (1ll << 31));
  GenArgs a{(const char*)dy, lddy, N, P, Q, Cout, H, W, (const char*)wt, C, R, S, stride, pad, 1, nullptr, (char*)dx,
            lddx, accumulate};
  hipStream_t st = (hipStream_t)stream;
  return dtype == DG_BF16 ? launch_gen<bf16>(a, st) : dtype == DG_F16 ? launch_gen<f16>(a, st) : launch_gen<float>(a, st);
}

extern "C" int64_t dg_conv2d_wgrad_workspace(int dtype, int N, int P, int Q, int C, int Cout, int R, int S) {
  return dg_conv_wgrad_workspace(dtype, N, P, Q, C, Cout, R, S);
}

extern "C" int dg_conv2d_wgrad(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, const void* dy,
                               int64_t lddy, int Cout, int R, int S, int stride, int pad, float* dw, void* workspace,
                               int64_t ws_bytes, int accumulate, const float* xamax, const float* dyamax,
                               void* stream) {
  DG_REQUIRE(x && dy && dw && workspace && stride >= 1 && pad >= 0);
  DG_REQUIRE(dtype == DG_F32 || DG_IS16(dtype));
  DG_SUPPORTED(Cout % 64 == 0 && C % 64 == 0);
  DG_REQUIRE(ldx % 8 == 0 && lddy % 8 == 0 && ldx >= C && lddy >= Cout);
  const int P = conv_out(H, R, stride, pad), Q = conv_out(W, S, stride, pad);
  DG_REQUIRE(P > 0 && Q > 0);
  const int64_t need = dg_conv_wgrad_workspace(dtype, N, P, Q, C, Cout, R, S);
  DG_REQUIRE(ws_bytes >= need);
  WgPlan p = DG_IS16(dtype) ? wg_plan<bf16>(N, P, Q, C, Cout, R, S) : wg_plan<float>(N, P, Q, C, Cout, R, S);
  DG_SUPPORTED((((long long)N * H * W - 1) * ldx + C) * (DG_IS16(dtype) ? 2 : 4) < (1ll << 31));
  DG_SUPPORTED((long long)p.pps * lddy * 4 < (1ll << 31));
  WgArgs a{(const char*)x, ldx, N, H, W, C, (const char*)dy, lddy, Cout, R, S, pad, (float*)workspace, p.splits, p.pps,
           stride, P, Q, 1};
  a.xam = (const unsigned*)xamax;
  a.dyam = (const unsigned*)dyamax;
  hipStream_t st = (hipStream_t)stream;
  unsigned* hslots = dtype == DG_F32 ? (unsigned*)((char*)workspace + need - wg_amax_bytes(C, Cout)) : nullptr;
  return dtype == DG_BF16 ? launch_wgrad<bf16>(a, dw, accumulate, st) : dtype == DG_F16 ? launch_wgrad<f16>(a, dw, accumulate, st) : launch_wgrad<float>(a, dw, accumulate, st, hslots);
}


extern "C" int dg_im2col_c3(int dtype, const float* img, int N, int H, int W, int R, int S, int stride, int pad,
                            int Kpad, void* out, void* stream) {
  DG_REQUIRE(img && out && N > 0 && H > 0 && W > 0 && R > 0 && S > 0 && stride >= 1 && Kpad >= R * S * 3);
  const int P = conv_out(H, R, stride, pad), Q = conv_out(W, S, stride, pad);
  DG_REQUIRE(P > 0 && Q > 0);
  DG_SUPPORTED(Kpad % 8 == 0 && (long long)N * P * Q < (1LL << 31));
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)N * P * Q * (Kpad / (DG_IS16(dtype) ? 8 : 4));
  if (im2col_lds_ok(R, S, stride, Kpad) && (dtype == DG_BF16 || dtype == DG_F16 || dtype == DG_F32)) {
    const dim3 g((unsigned)((long long)N * P * dg_cdiv(Q, I2C_QB)));
    if (dtype == DG_BF16)
      hipLaunchKernelGGL(im2col_c3_lds_kernel<bf16>, g, dim3(256), 0, st, img, N, H, W, R, S, stride, pad, P, Q, Kpad,
                         (bf16*)out);
    else if (dtype == DG_F16)
      hipLaunchKernelGGL(im2col_c3_lds_kernel<f16>, g, dim3(256), 0, st, img, N, H, W, R, S, stride, pad, P, Q, Kpad,
                         (f16*)out);
    else
      hipLaunchKernelGGL(im2col_c3_lds_kernel<float>, g, dim3(256), 0, st, img, N, H, W, R, S, stride, pad, P, Q, Kpad,
                         (float*)out);
  } else if (dtype == DG_BF16)
    hipLaunchKernelGGL(im2col_c3_ex_kernel<bf16>, dim3(grid_for(total, 256, 1 << 20)), dim3(256), 0, st, img, N, H, W,
                       R, S, stride, pad, P, Q, Kpad, (bf16*)out);
  else if (dtype == DG_F16)
    hipLaunchKernelGGL(im2col_c3_ex_kernel<f16>, dim3(grid_for(total, 256, 1 << 20)), dim3(256), 0, st, img, N, H, W,
                       R, S, stride, pad, P, Q, Kpad, (f16*)out);
  else if (dtype == DG_F32)
    hipLaunchKernelGGL(im2col_c3_ex_kernel<float>, dim3(grid_for(total, 256, 1 << 20)), dim3(256), 0, st, img, N, H,
                       W, R, S, stride, pad, P, Q, Kpad, (float*)out);
  else
    return DG_ERR_INVALID;
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_unpack_c3(const float* dwcol, int Cout, int R, int S, int Kpad, float* dw, int accumulate,
                            void* stream) {
  DG_REQUIRE(dwcol && dw && Cout > 0 && Kpad >= R * S * 3);
  hipLaunchKernelGGL(unpack_c3_ex_kernel, dim3(grid_for((long long)Cout * 3 * R * S)), dim3(256), 0,
                     (hipStream_t)stream, dwcol, Cout, R, S, Kpad, dw, accumulate);
  DG_CHECK_LAUNCH();
  return DG_OK;
}
