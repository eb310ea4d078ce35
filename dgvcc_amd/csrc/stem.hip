// First VGG16-BN layer (features[0:3] = Conv2d(3, 64, 3, pad 1) + BatchNorm2d +
// ReLU, models/models.py:35-36) fused for the bf16 perf path.
//
// The generic route materialised a [N*H*W][64] im2col buffer (27 taps padded to
// 64) and ran the K=64 GEMM on it, then read the conv output again for the BN
// statistics: ~3.5 GB of HBM traffic per 16 frames at 768x1024 for 0.1 TFLOP.
// Here:
//   forward  stem_fwd_kernel  gathers the 27 taps straight from the NCHW f32
//            image into MFMA B fragments (v_mfma_f32_16x16x32_bf16, K = 27 -> 32),
//            adds the bias, writes z (bf16 NHWC) and keeps per-channel shifted
//            sums of the stored values -> per-block (n, mean, M2) partials;
//            bn_part_finalize merges them (Chan) in double.
//   backward stem_bwd_kernel recomputes dz = BN/ReLU backward (the same float
//            arithmetic as bn_bwd_apply in norm.hip) from g and z, stages dz and
//            the image im2col tile in LDS and accumulates dW = dz^T . col on MFMA
//            (transposed ds_read_b64_tr_b16 fragments).  dz never reaches HBM
//            (the first layer has no input gradient).
#include "dg_common.h"
#include <algorithm>
#include <cstdlib>

extern "C" int dg_bn_bwd_finalize_part(const float* part, int nblk, int M, int C, const float* gamma,
                                       const float* save_invstd, float* dgamma, float* dbeta, float* dbias,
                                       float* coef, void* stream);  // norm.hip

namespace {

constexpr int SNT = 256;     // 4 waves
constexpr int SCO = 64;      // output channels of the stem
constexpr int SK = 32;       // 27 taps padded to one bf16 MFMA k-step

__device__ __forceinline__ unsigned short bfbits(float x) { return f2bf(x); }

// Wave-independent row segments (W % 64 == 0): a segment is 64 consecutive
// pixels of one image row.  The 3 channels x 3 rows x 66 columns it needs are
// loaded coalesced (one float per lane and row, prefetched a segment ahead) and
// staged in the wave's own LDS slice as bf16; B fragments are then gathered from
// LDS.  The output fragment (16 px x 64 co) is transposed through LDS so every
// global store is a full 16-B lane / 1-KB wave write.
constexpr int TROW = 72;                       // staged image row: 66 used (q0-1 .. q0+64)
constexpr int T_BYTES = 9 * TROW * 2;          // [c][r][TROW] bf16
constexpr int O_BYTES = 16 * 128;              // [16 px][64 co] bf16, 16-B chunks XOR-swizzled by row
constexpr int FW_LDS = T_BYTES + O_BYTES;

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// MODE 0: write z and the BN statistics partials; 1: statistics only (z is recomputed by
// its consumers instead of stored); 2: y = relu(bn(z)) with z recomputed (the stored bf16 z
// value, then dg_bn_apply's arithmetic) written to `z`, no statistics; 3: the BN-backward
// partial sums of g (sum g', sum g' xhat, sum xhat; g' = g relu'(bn(z))) with z recomputed:
// plain per-block sums for bn_bwd_finalize.
struct StemBn {
  const float *sc, *sf, *mu, *is;  // BN scale/shift and saved mean/invstd
  const bf16* g;                   // MODE 3: gradient of y
  long long ldg;
};

template <int MODE>
__global__ __launch_bounds__(SNT, 2) void stem_fwd_kernel(const float* __restrict__ img, int H, int W,
                                                          const bf16* __restrict__ wp, const float* __restrict__ bias,
                                                          bf16* __restrict__ z, long long ldz, long long nseg,
                                                          float* __restrict__ part, StemBn bn) {
  __shared__ __attribute__((aligned(16))) char smem[4 * FW_LDS];
  __shared__ float sh[4][3][SCO];
  __shared__ __attribute__((aligned(16))) float bnp[4][SCO];  // MODE 2/3: scale, shift, mean, invstd
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int h = lane >> 4, col = lane & 15;
  char* T = smem + wid * FW_LDS;
  if constexpr (MODE >= 2) {
    const int k = threadIdx.x / SCO, c = threadIdx.x - k * SCO;  // 256 threads = 4 x 64
    const float* src = k == 0 ? bn.sc : k == 1 ? bn.sf : k == 2 ? bn.mu : bn.is;
    bnp[k][c] = src ? src[c] : 0.f;
    __syncthreads();
  }
  char* O = T + T_BYTES;
  const int spr = W / 64;  // segments per image row
  // LDS byte offsets of this lane's 8 taps (k = 8h + j) relative to pixel column x
  int toff[8];
  unsigned kmask = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * h + j;
    const int t = k / 3, c = k - 3 * t, r = t / 3, s2 = t - 3 * r;
    toff[j] = ((c * 3 + r) * TROW + s2) * 2;
    if (k < 27) kmask |= 1u << j;
  }
  u4v wa[4];
  float bs[4][4];
#pragma unroll
  for (int cf = 0; cf < 4; ++cf) {
    wa[cf] = *(const u4v*)(wp + (16 * cf + col) * SK + 8 * h);
#pragma unroll
    for (int i = 0; i < 4; ++i) bs[cf][i] = bias ? bias[16 * cf + 4 * h + i] : 0.f;
  }
  float K[16], S1[16], S2[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) { K[e] = 0.f; S1[e] = 0.f; S2[e] = 0.f; }

  float raw[9], rawt[9];
  auto gload = [&](long long seg) {
    const int row_id = (int)(seg / spr);            // n*H + p
    const int q0 = (int)(seg - (long long)row_id * spr) * 64;
    const int n = row_id / H, p = row_id - n * H;
    const int qa = q0 - 1 + lane, qb = q0 + 63 + lane;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int pr = p + r - 1;
        const bool rok = (unsigned)pr < (unsigned)H;
        const float* src = img + ((long long)(n * 3 + c) * H + pr) * W;
        raw[c * 3 + r] = (rok && qa >= 0) ? src[qa] : 0.f;
        rawt[c * 3 + r] = (rok && lane < 2 && qb < W) ? src[qb] : 0.f;
      }
  };
  long long seg = (long long)blockIdx.x * 4 + wid;
  const long long sstride = (long long)gridDim.x * 4;
  if (seg < nseg) gload(seg);
  long long nloc = 0;
  bool first = true;
  for (; seg < nseg; seg += sstride) {
    // stage the image rows (bf16), then prefetch the next segment's
    unsigned short* Ts = (unsigned short*)T;
#pragma unroll
    for (int e = 0; e < 9; ++e) {
      Ts[e * TROW + lane] = bfbits(raw[e]);
      if (lane < 2) Ts[e * TROW + 64 + lane] = bfbits(rawt[e]);
    }
    lds_fence();
    if (seg + sstride < nseg) gload(seg + sstride);
    const long long m0 = seg * 64;
    // MODE 3 keeps 3 x 16 accumulators and the pixel group's g live: the pixel-group loop
    // stays rolled there (fully unrolled it spills)
    constexpr int PFU = MODE == 3 ? 1 : 4;
#pragma unroll PFU
    for (int pf = 0; pf < 4; ++pf) {
      u2v graw[4];  // MODE 3: this pixel group's g, 4 loads issued before the first use
      if constexpr (MODE == 3) {
#pragma unroll
        for (int cf = 0; cf < 4; ++cf)
          graw[cf] = *(const u2v*)(bn.g + (m0 + 16 * pf + col) * bn.ldg + 16 * cf + 4 * h);
      }
      const int x2 = (16 * pf + col) * 2;
      unsigned short v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (kmask >> j) & 1 ? *(const unsigned short*)(T + toff[j] + x2) : 0;
      const u4v b = u4v{v[0] | ((unsigned)v[1] << 16), v[2] | ((unsigned)v[3] << 16), v[4] | ((unsigned)v[5] << 16),
                        v[6] | ((unsigned)v[7] << 16)};
      f4v acc[4];
#pragma unroll
      for (int cf = 0; cf < 4; ++cf)
        acc[cf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(s8v, wa[cf]), __builtin_bit_cast(s8v, b),
                                                          f4v{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
      for (int cf = 0; cf < 4; ++cf) {
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = bf2f(bfbits(acc[cf][i] + bs[cf][i]));  // the stored value
        const int cb = 16 * cf + 4 * h;
        if constexpr (MODE == 2) {  // dg_bn_apply: relu(fmaf(z, scale, shift))
          const f4v sc4 = *(const f4v*)&bnp[0][cb], sf4 = *(const f4v*)&bnp[1][cb];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float t = fmaf(o[i], sc4[i], sf4[i]);
            o[i] = t > 0.f ? t : 0.f;
          }
        }
        if constexpr (MODE == 0 || MODE == 2) {
          const int chunk = 2 * cf + (h >> 1);
          *(u2v*)(O + col * 128 + ((chunk ^ (col & 7)) << 4) + (h & 1) * 8) =
              u2v{pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3])};
        }
        if constexpr (MODE == 0 || MODE == 1) {
          if (first && pf == 0) {  // per-channel shift: the wave's first pixel (lane col 0 of its group)
#pragma unroll
            for (int i = 0; i < 4; ++i) K[cf * 4 + i] = __shfl(o[i], lane & 48, 64);
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float d = o[i] - K[cf * 4 + i];
            S1[cf * 4 + i] += d;
            S2[cf * 4 + i] = fmaf(d, d, S2[cf * 4 + i]);
          }
        }
        if constexpr (MODE == 3) {  // bn_bwd_load + bn_bwd_partial of norm.hip (act = relu, no dropout)
          const u2v gr = graw[cf];
          const float gv[4] = {__uint_as_float(gr[0] << 16), __uint_as_float(gr[0] & 0xffff0000u),
                               __uint_as_float(gr[1] << 16), __uint_as_float(gr[1] & 0xffff0000u)};
          const f4v sc4 = *(const f4v*)&bnp[0][cb], sf4 = *(const f4v*)&bnp[1][cb];
          const f4v mu4 = *(const f4v*)&bnp[2][cb], is4 = *(const f4v*)&bnp[3][cb];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float gg = gv[i];
            if (!(fmaf(o[i], sc4[i], sf4[i]) > 0.f)) gg = 0.f;
            const float xh = (o[i] - mu4[i]) * is4[i];
            S1[cf * 4 + i] += gg;
            S2[cf * 4 + i] = fmaf(gg, xh, S2[cf * 4 + i]);
            K[cf * 4 + i] += xh;
          }
        }
      }
      if constexpr (MODE == 0 || MODE == 2) {
        lds_fence();
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int row = (lane >> 3) + 8 * u, chunk = lane & 7;
          const u4v ov = *(const u4v*)(O + row * 128 + ((chunk ^ (row & 7)) << 4));
          *(u4v*)(z + (m0 + 16 * pf + row) * ldz + chunk * 8) = ov;
        }
      }
    }
    first = false;
    nloc += 64;
  }
  if constexpr (MODE == 2) return;
  // reduce over the 16 pixel lanes of each group
#pragma unroll
  for (int e = 0; e < 16; ++e) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      S1[e] += __shfl_xor(S1[e], o, 64);
      S2[e] += __shfl_xor(S2[e], o, 64);
      if constexpr (MODE == 3) K[e] += __shfl_xor(K[e], o, 64);
    }
  }
  if constexpr (MODE == 3) {  // plain sums: 4 waves in a fixed order -> one part row per block
    if (col == 0) {
#pragma unroll
      for (int cf = 0; cf < 4; ++cf)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 16 * cf + 4 * h + i, e = cf * 4 + i;
          sh[wid][0][c] = S1[e];
          sh[wid][1][c] = S2[e];
          sh[wid][2][c] = K[e];
        }
    }
    __syncthreads();
    if (threadIdx.x < 3 * SCO) {
      const int k = threadIdx.x / SCO, c = threadIdx.x - k * SCO;
      part[(long long)blockIdx.x * 3 * SCO + k * SCO + c] = sh[0][k][c] + sh[1][k][c] + sh[2][k][c] + sh[3][k][c];
    }
    return;
  }
  if (col == 0) {
#pragma unroll
    for (int cf = 0; cf < 4; ++cf)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 16 * cf + 4 * h + i, e = cf * 4 + i;
        const float nn = (float)nloc;
        sh[wid][0][c] = nn;
        sh[wid][1][c] = nloc ? K[e] + S1[e] / nn : 0.f;
        sh[wid][2][c] = nloc ? fmaxf(S2[e] - S1[e] * S1[e] / nn, 0.f) : 0.f;
      }
  }
  __syncthreads();
  if (threadIdx.x < SCO) {  // Chan merge of the 4 waves
    const int c = threadIdx.x;
    float n = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float nb = sh[w][0][c];
      if (nb == 0.f) continue;
      const float mb = sh[w][1][c];
      const float nt = n + nb;
      const float d = mb - mean;
      mean += d * (nb / nt);
      m2 += sh[w][2][c] + d * d * (n * nb / nt);
      n = nt;
    }
    float* o = part + (long long)blockIdx.x * 3 * SCO;
    o[c] = n;
    o[SCO + c] = mean;
    o[2 * SCO + c] = m2;
  }
}

// fp32 first layer forward: exact f32 FMAs on the VALU (27 MACs per output; 0.1 TFLOP per 16
// frames at 768x1024 is below the VALU's ~1 ms, and an MFMA split would need 6 products per
// f32 product), replacing the generic route's [N*H*W][64] f32 im2col buffer, its K = 64
// GEMM and the separate BN statistics pass over z.  Wave-independent 64-pixel row segments,
// lane = pixel: the 27 taps are loaded straight from the NCHW image (prefetched a segment
// ahead), the filter wk[27][64] is wave-uniform (scalar loads), the 64 channel results go
// through the wave's LDS tile [64 px][64 co] (16-B chunks XOR-swizzled by pixel) so the z
// stores are 1-KB wave writes, and the statistics read the tile back with lane = channel
// (shifted sums, then the Chan merge of stem_fwd_kernel's epilogue: same part rows).
constexpr int F32_TILE = 64 * 16;  // f4v chunks per wave tile (16 KB)

__global__ __launch_bounds__(SNT, 2) void stem_fwd_f32_kernel(const float* __restrict__ img, int H, int W,
                                                              const float* __restrict__ wk,
                                                              const float* __restrict__ bias, float* __restrict__ z,
                                                              long long ldz, long long nseg, float* __restrict__ part) {
  __shared__ f4v tile[4 * F32_TILE];
  __shared__ float sh[4][3][SCO];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  f4v* O = tile + wid * F32_TILE;
  const int spr = W / 64;
  // bias in the store / statistics phases, where lanes own channels
  const int cq = lane >> 2, ci = lane & 3;
  const f4v b4 = bias ? *(const f4v*)(bias + 4 * (lane & 15)) : f4v{0.f, 0.f, 0.f, 0.f};
  const float b1 = bias ? bias[lane] : 0.f;
  float xv[27];
  auto gload = [&](long long seg) {
    const int row_id = (int)(seg / spr);  // n*H + p
    const int q = (int)(seg - (long long)row_id * spr) * 64 + lane;
    const int n = row_id / H, p = row_id - n * H;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int pr = p + r - 1;
        const bool rok = (unsigned)pr < (unsigned)H;
        const float* src = img + ((long long)(n * 3 + c) * H + (rok ? pr : 0)) * W + q;
        const int e = (c * 3 + r) * 3;
        xv[e] = (rok && q >= 1) ? src[-1] : 0.f;
        xv[e + 1] = rok ? src[0] : 0.f;
        xv[e + 2] = (rok && q + 1 < W) ? src[1] : 0.f;
      }
  };
  float Ksh = 0.f, S1 = 0.f, S2 = 0.f;
  long long nloc = 0;
  long long seg = (long long)blockIdx.x * 4 + wid;
  const long long sstride = (long long)gridDim.x * 4;
  if (seg < nseg) gload(seg);
  for (; seg < nseg; seg += sstride) {
    lds_fence();  // the previous segment's tile reads are done before it is overwritten
    // 16 channels per pass (rolled): 16 accumulators, the pass's filter slice [27][16] is
    // wave-uniform and arrives through scalar loads one 16-float row per tap
#pragma unroll 1
    for (int cc = 0; cc < 4; ++cc) {
      const float* w = wk + 16 * cc;
      float acc[16];
#pragma unroll
      for (int co = 0; co < 16; ++co) acc[co] = 0.f;
      // one tap's 16 weights in flight ahead of its FMAs; the opaque address keeps the compiler
      // from hoisting all 432 scalar loads of the pass (which spills the SGPR file)
      float wc[16], wn[16];
#pragma unroll
      for (int co = 0; co < 16; ++co) wc[co] = w[co];
#pragma unroll
      for (int k = 0; k < 27; ++k) {
        if (k + 1 < 27) {
          int off = (k + 1) * SCO;
          asm volatile("" : "+s"(off));  // opaque offset: the load cannot move above this tap
#pragma unroll
          for (int co = 0; co < 16; ++co) wn[co] = w[off + co];
        }
        const float xk = xv[k];
#pragma unroll
        for (int co = 0; co < 16; ++co) acc[co] = fmaf(xk, wc[co], acc[co]);
#pragma unroll
        for (int co = 0; co < 16; ++co) wc[co] = wn[co];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        O[lane * 16 + ((4 * cc + j) ^ (lane & 15))] = f4v{acc[4 * j], acc[4 * j + 1], acc[4 * j + 2], acc[4 * j + 3]};
    }
    if (seg + sstride < nseg) gload(seg + sstride);
    lds_fence();
    const long long m0 = seg * 64;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int row = 4 * u + (lane >> 4), ch = lane & 15;
      const f4v v = O[row * 16 + (ch ^ (row & 15))];
      *(f4v*)(z + (m0 + row) * ldz + 4 * ch) = f4v{v[0] + b4[0], v[1] + b4[1], v[2] + b4[2], v[3] + b4[3]};
    }
    // statistics of the stored values (the same fp32 add), lane = channel
    const float* Of = (const float*)O;
    if (nloc == 0) Ksh = Of[cq * 4 + ci] + b1;  // pixel 0: chunk cq ^ 0
#pragma unroll 8
    for (int px = 0; px < 64; ++px) {
      const float d = (Of[(px * 16 + (cq ^ (px & 15))) * 4 + ci] + b1) - Ksh;
      S1 += d;
      S2 = fmaf(d, d, S2);
    }
    nloc += 64;
  }
  {
    const float nn = (float)nloc;
    sh[wid][0][lane] = nn;
    sh[wid][1][lane] = nloc ? Ksh + S1 / nn : 0.f;
    sh[wid][2][lane] = nloc ? fmaxf(S2 - S1 * S1 / nn, 0.f) : 0.f;
  }
  __syncthreads();
  if (threadIdx.x < SCO) {  // Chan merge of the 4 waves
    const int c = threadIdx.x;
    float n = 0.f, mean = 0.f, m2 = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float nb = sh[w][0][c];
      if (nb == 0.f) continue;
      const float mb = sh[w][1][c];
      const float nt = n + nb;
      const float d = mb - mean;
      mean += d * (nb / nt);
      m2 += sh[w][2][c] + d * d * (n * nb / nt);
      n = nt;
    }
    float* o = part + (long long)blockIdx.x * 3 * SCO;
    o[c] = n;
    o[SCO + c] = mean;
    o[2 * SCO + c] = m2;
  }
}

// Backward, wave-independent 32-pixel row segments: dW[co][k] = sum_px dz[px][co] col[px][k].
// Per wave LDS: dz tile [32 px][64 co] bf16 (128-B rows, read transposed) and the
// transposed im2col tile colT[32 k][32 px] bf16 (64-B rows; rows 27..31 stay zero).
// Lane roles: dz for channels 8*(lane&7).. of pixels (lane>>3) + 8u; colT rows
// k = 2i + (lane>>5) at pixel lane&31.  Loads are prefetched a segment ahead.
// RECOMP = 1: z is not read from HBM but recomputed from the staged im2col tile (the same
// MFMA on the same bf16 operands as stem_fwd_kernel, so the same bits), transposed through
// a third per-wave LDS tile into the dz lane layout.
constexpr int CTS = 72;  // colT row stride (B): the 4 k-groups of a B-fragment gather hit distinct banks
constexpr int BDZ = 32 * 128, BCOL = 32 * CTS, BZT = 32 * 128;

template <int RECOMP>
__global__ __launch_bounds__(SNT, 2) void stem_bwd_kernel(
    const float* __restrict__ img, int H, int W, const bf16* __restrict__ g, long long ldg, const bf16* __restrict__ z,
    long long ldz, const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ scale,
    const float* __restrict__ shift, const float* __restrict__ coef, long long nseg, float* __restrict__ slab,
    const bf16* __restrict__ wpk, const float* __restrict__ bias) {
  constexpr int BW_LDS = BDZ + BCOL + (RECOMP ? BZT : 0);
  __shared__ __attribute__((aligned(16))) char smem[4 * BW_LDS];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  char* DZ = smem + wid * BW_LDS;
  char* CT = DZ + BDZ;
  char* ZT = CT + BCOL;  // RECOMP: z tile [32 px][64 co] bf16
  u4v wa[4];             // RECOMP: filter fragments (A operand) as stem_fwd_kernel
  __shared__ __attribute__((aligned(16))) float bsl[SCO];  // RECOMP: conv bias (LDS: registers are full)
  if constexpr (RECOMP) {
    const int col = lane & 15, hh = lane >> 4;
#pragma unroll
    for (int cf = 0; cf < 4; ++cf) wa[cf] = *(const u4v*)(wpk + (16 * cf + col) * SK + 8 * hh);
    if (threadIdx.x < SCO) bsl[threadIdx.x] = bias ? bias[threadIdx.x] : 0.f;
    __syncthreads();
  }
  const int spr = W / 32;
  const int c0 = (lane & 7) * 8;
  float sc[8], sf[8], mu[8], is[8], k1[8], k2[8], k3[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = scale[c0 + e]; sf[e] = shift[c0 + e]; mu[e] = mean[c0 + e]; is[e] = invstd[c0 + e];
    k1[e] = coef[c0 + e]; k2[e] = coef[SCO + c0 + e]; k3[e] = coef[2 * SCO + c0 + e];
  }
  // colT rows of this lane: k = 2i + (lane>>5), i = 0..13 (k = 27 -> zero); px = lane & 31
  const int half = lane >> 5, xq = lane & 31;
  for (int r = 28 + half; r < 32; r += 2) *(unsigned short*)(CT + r * CTS + xq * 2) = 0;

  struct Regs {
    u4v gr[4], zr[4];
    float cv[14];
  };
  auto gload = [&](Regs& R, long long seg) {
    const int row_id = (int)(seg / spr);
    const int q0 = (int)(seg - (long long)row_id * spr) * 32;
    const int n = row_id / H, p = row_id - n * H;
    const long long m0 = (long long)row_id * W + q0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long m = m0 + (lane >> 3) + 8 * u;
      R.gr[u] = *(const u4v*)(g + m * ldg + c0);
      if constexpr (!RECOMP) R.zr[u] = *(const u4v*)(z + m * ldz + c0);
    }
#pragma unroll
    for (int i = 0; i < 14; ++i) {
      const int k = 2 * i + half;
      const int t = k / 3, c = k - 3 * t, r = t / 3, s2 = t - 3 * r;
      const int pr = p + r - 1, qq = q0 + xq + s2 - 1;
      const bool in = k < 27 && (unsigned)pr < (unsigned)H && (unsigned)qq < (unsigned)W;
      R.cv[i] = in ? img[((long long)(n * 3 + c) * H + pr) * W + qq] : 0.f;
    }
  };
  f4v acc[4][2];
#pragma unroll
  for (int cf = 0; cf < 4; ++cf) acc[cf][0] = acc[cf][1] = f4v{0.f, 0.f, 0.f, 0.f};
  const int gq = lane >> 4, q4 = (lane & 15) >> 2, p4 = lane & 3, li = lane & 15;
  auto process = [&](const Regs& R) {
    u4v zrow[4];
    if constexpr (RECOMP) {
      // im2col tile first; z = W . colT on MFMA (B fragments gathered as stem_fwd_kernel does)
#pragma unroll
      for (int i = 0; i < 14; ++i) *(unsigned short*)(CT + (2 * i + half) * CTS + xq * 2) = bfbits(R.cv[i]);
      lds_fence();
      const int col = lane & 15, hh = lane >> 4;
#pragma unroll
      for (int pb = 0; pb < 2; ++pb) {
        unsigned short v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = *(const unsigned short*)(CT + (8 * hh + j) * CTS + (16 * pb + col) * 2);
        const u4v b = u4v{v[0] | ((unsigned)v[1] << 16), v[2] | ((unsigned)v[3] << 16),
                          v[4] | ((unsigned)v[5] << 16), v[6] | ((unsigned)v[7] << 16)};
#pragma unroll
        for (int cf = 0; cf < 4; ++cf) {
          const f4v a4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(s8v, wa[cf]),
                                                                 __builtin_bit_cast(s8v, b), f4v{0.f, 0.f, 0.f, 0.f},
                                                                 0, 0, 0);
          const f4v b4 = *(const f4v*)&bsl[16 * cf + 4 * hh];
          float o[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = bf2f(bfbits(a4[i] + b4[i]));  // stem_fwd's stored value
          const int zr = 16 * pb + col, chunk = 2 * cf + (hh >> 1);  // 16-B chunks XOR-swizzled by row
          *(u2v*)(ZT + zr * 128 + ((chunk ^ (zr & 7)) << 4) + (hh & 1) * 8) =
              u2v{pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3])};
        }
      }
      lds_fence();
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int zr = (lane >> 3) + 8 * u, chunk = lane & 7;
        zrow[u] = *(const u4v*)(ZT + zr * 128 + ((chunk ^ (zr & 7)) << 4));
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) zrow[u] = R.zr[u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float gv[8], zv[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        gv[2 * i] = __uint_as_float(R.gr[u][i] << 16); gv[2 * i + 1] = __uint_as_float(R.gr[u][i] & 0xffff0000u);
        zv[2 * i] = __uint_as_float(zrow[u][i] << 16); zv[2 * i + 1] = __uint_as_float(zrow[u][i] & 0xffff0000u);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {  // bn_bwd_load + bn_bwd_apply of norm.hip (act = relu, no dropout)
        if (!(fmaf(zv[e], sc[e], sf[e]) > 0.f)) gv[e] = 0.f;
        const float xh = (zv[e] - mu[e]) * is[e];
        gv[e] = k1[e] * gv[e] - k2[e] * xh - k3[e];
      }
      const int px = (lane >> 3) + 8 * u;
      *(u4v*)(DZ + px * 128 + c0 * 2) =
          u4v{pack_bf2(gv[0], gv[1]), pack_bf2(gv[2], gv[3]), pack_bf2(gv[4], gv[5]), pack_bf2(gv[6], gv[7])};
    }
    if constexpr (!RECOMP) {
#pragma unroll
      for (int i = 0; i < 14; ++i) *(unsigned short*)(CT + (2 * i + half) * CTS + xq * 2) = bfbits(R.cv[i]);
    }
    lds_fence();
    // A = dz^T (transposed reads): logical k = 8*gq + j <-> pixel 4*gq + (j&3) + 16*(j>>2)
    s8v bfv[2];
#pragma unroll
    for (int kf = 0; kf < 2; ++kf) {
      const char* rp = CT + (16 * kf + li) * CTS;
      const u2v lo = *(const u2v*)(rp + 8 * gq), hi = *(const u2v*)(rp + 32 + 8 * gq);
      bfv[kf] = __builtin_bit_cast(s8v, u4v{lo[0], lo[1], hi[0], hi[1]});
    }
#pragma unroll
    for (int cf = 0; cf < 4; ++cf) {
      const int ca = (16 * cf + 4 * p4) * 2;
      s4v alo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DG_LDS s4v*)(DZ + (4 * gq + q4) * 128 + ca));
      s4v ahi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((DG_LDS s4v*)(DZ + (16 + 4 * gq + q4) * 128 + ca));
      const s8v af = s8v{alo[0], alo[1], alo[2], alo[3], ahi[0], ahi[1], ahi[2], ahi[3]};
#pragma unroll
      for (int kf = 0; kf < 2; ++kf) acc[cf][kf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfv[kf], acc[cf][kf], 0, 0, 0);
    }
  };
  // two register sets: segment i+1's loads are issued before segment i is processed
  Regs RA, RB;
  long long seg = (long long)blockIdx.x * 4 + wid;
  const long long sstride = (long long)gridDim.x * 4;
  if (seg < nseg) gload(RA, seg);
  for (; seg < nseg; seg += 2 * sstride) {
    const long long s1 = seg + sstride;
    if (s1 < nseg) gload(RB, s1);
    process(RA);
    if (s1 >= nseg) break;
    if (s1 + sstride < nseg) gload(RA, s1 + sstride);
    process(RB);
  }
  // combine the 4 waves in a fixed order (deterministic), then one slab row per block
  __syncthreads();
  float* red = (float*)smem;  // [64 co][32 k]
  for (int w = 0; w < 4; ++w) {
    if (wid == w) {
#pragma unroll
      for (int cf = 0; cf < 4; ++cf)
#pragma unroll
        for (int kf = 0; kf < 2; ++kf)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float* d = red + (16 * cf + 4 * gq + i) * SK + 16 * kf + li;
            *d = (w == 0 ? 0.f : *d) + acc[cf][kf][i];
          }
    }
    __syncthreads();
  }
  float* o = slab + (long long)blockIdx.x * SCO * SK;
  for (int e = threadIdx.x; e < SCO * SK; e += SNT) o[e] = red[e];
}

// fp32 backward of the first layer: dz = BN/ReLU backward of (g, z) (bn_bwd_apply's arithmetic)
// and dW[co][k] = sum_px dz[px][co] col[px][k] on v_mfma_f32_16x16x4_f32 (exact f32 products),
// without the dz tensor or the im2col buffer in HBM.  Wave-independent 32-pixel row segments;
// per wave LDS: dz [32 px][64 co] f32 (row stride 80 floats: the 4 pixel rows of an A read hit
// distinct banks) and colT [32 k][32 px] f32 (stride 36: the 16 k rows x 4 pixels of a B read
// hit distinct banks; rows 27..31 zero).  The next segment's g, z and taps are loaded while
// this one's MFMAs run.  Output: one slab row [64][32] per block (stem_wgrad_reduce order
// k = (r*3+s)*3+c), combined over the 4 waves in a fixed order.
constexpr int F_DZS = 80, F_CTS = 36;
constexpr int F_BW = (32 * F_DZS + 32 * F_CTS) * 4;

__global__ __launch_bounds__(SNT, 2) void stem_bwd_f32_kernel(
    const float* __restrict__ img, int H, int W, const float* __restrict__ g, long long ldg,
    const float* __restrict__ z, long long ldz, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ scale, const float* __restrict__ shift, const float* __restrict__ coef, long long nseg,
    float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) char smem[4 * F_BW];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float* DZ = (float*)(smem + wid * F_BW);
  float* CT = DZ + 32 * F_DZS;
  const int spr = W / 32;
  const int c0 = (lane & 15) * 4;  // this lane's 4 channels in the dz phase
  float sc[4], sf[4], mu[4], is[4], k1[4], k2[4], k3[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    sc[e] = scale[c0 + e]; sf[e] = shift[c0 + e]; mu[e] = mean[c0 + e]; is[e] = invstd[c0 + e];
    k1[e] = coef[c0 + e]; k2[e] = coef[SCO + c0 + e]; k3[e] = coef[2 * SCO + c0 + e];
  }
  const int half = lane >> 5, xq = lane & 31;
  for (int r = 27 + half; r < 32; r += 2) CT[r * F_CTS + xq] = 0.f;
  f4v gr[8], zr[8];
  float cv[14];
  auto gload = [&](long long seg) {
    const int row_id = (int)(seg / spr);
    const int q0 = (int)(seg - (long long)row_id * spr) * 32;
    const int n = row_id / H, p = row_id - n * H;
    const long long m0 = (long long)row_id * W + q0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long long m = m0 + (lane >> 4) + 4 * u;
      gr[u] = *(const f4v*)(g + m * ldg + c0);
      zr[u] = *(const f4v*)(z + m * ldz + c0);
    }
#pragma unroll
    for (int i = 0; i < 14; ++i) {
      const int k = 2 * i + half;
      const int t = k / 3, c = k - 3 * t, r = t / 3, s2 = t - 3 * r;
      const int pr = p + r - 1, qq = q0 + xq + s2 - 1;
      const bool in = k < 27 && (unsigned)pr < (unsigned)H && (unsigned)qq < (unsigned)W;
      cv[i] = in ? img[((long long)(n * 3 + c) * H + pr) * W + qq] : 0.f;
    }
  };
  f4v acc[4][2];
#pragma unroll
  for (int cf = 0; cf < 4; ++cf) acc[cf][0] = acc[cf][1] = f4v{0.f, 0.f, 0.f, 0.f};
  const int mrow = lane & 15, kq = lane >> 4;  // MFMA operand roles: A[m][k], B[k][n]
  long long seg = (long long)blockIdx.x * 4 + wid;
  const long long sstride = (long long)gridDim.x * 4;
  if (seg < nseg) gload(seg);
  for (; seg < nseg; seg += sstride) {
    lds_fence();  // the previous segment's fragment reads are done before the tiles are overwritten
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      float dz[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // bn_bwd_load + bn_bwd_apply of norm.hip (act = relu, no dropout)
        float gv = gr[u][e];
        const float zv = zr[u][e];
        if (!(fmaf(zv, sc[e], sf[e]) > 0.f)) gv = 0.f;
        const float xh = (zv - mu[e]) * is[e];
        dz[e] = k1[e] * gv - k2[e] * xh - k3[e];
      }
      *(f4v*)(DZ + ((lane >> 4) + 4 * u) * F_DZS + c0) = f4v{dz[0], dz[1], dz[2], dz[3]};
    }
#pragma unroll
    for (int i = 0; i < 14; ++i)
      if (2 * i + half < 27) CT[(2 * i + half) * F_CTS + xq] = cv[i];
    if (seg + sstride < nseg) gload(seg + sstride);
    lds_fence();
#pragma unroll
    for (int s = 0; s < 8; ++s) {  // 4 pixels per MFMA k-step
      const int px = 4 * s + kq;
      float bv[2];
#pragma unroll
      for (int kf = 0; kf < 2; ++kf) bv[kf] = CT[(16 * kf + mrow) * F_CTS + px];
#pragma unroll
      for (int cf = 0; cf < 4; ++cf) {
        const float av = DZ[px * F_DZS + 16 * cf + mrow];
#pragma unroll
        for (int kf = 0; kf < 2; ++kf) acc[cf][kf] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[kf], acc[cf][kf], 0, 0, 0);
      }
    }
  }
  // combine the 4 waves in a fixed order (deterministic), then one slab row per block
  __syncthreads();
  float* red = (float*)smem;  // [64 co][32 k]
  for (int w = 0; w < 4; ++w) {
    if (wid == w) {
#pragma unroll
      for (int cf = 0; cf < 4; ++cf)
#pragma unroll
        for (int kf = 0; kf < 2; ++kf)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float* d = red + (16 * cf + 4 * kq + i) * SK + 16 * kf + mrow;
            *d = (w == 0 ? 0.f : *d) + acc[cf][kf][i];
          }
    }
    __syncthreads();
  }
  float* o = slab + (long long)blockIdx.x * SCO * SK;
  for (int e = threadIdx.x; e < SCO * SK; e += SNT) o[e] = red[e];
}

// out[rb][c] = sum of rows [rb*rpb, (rb+1)*rpb) of in[rows][cols]; grid (cols/256, ceil(rows/rpb)).
__global__ __launch_bounds__(SNT) void colsum_rows_kernel(const float* __restrict__ in, int rows, int cols, int rpb,
                                                          float* __restrict__ out) {
  const int c = blockIdx.x * SNT + threadIdx.x;
  if (c >= cols) return;
  const int r0 = blockIdx.y * rpb, r1 = min(rows, r0 + rpb);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += in[(long long)r * cols + c];
  out[(long long)blockIdx.y * cols + c] = s;
}

// dw[co][c][r][s] (torch layout) = sum_b slab[b][co][k], k = (r*3+s)*3+c; one block per co.
__global__ __launch_bounds__(SNT) void stem_wgrad_reduce(const float* __restrict__ slab, int nblk,
                                                         float* __restrict__ dw, int accumulate) {
  __shared__ float sh[8][SK];
  const int co = blockIdx.x, k = threadIdx.x & 31, rg = threadIdx.x >> 5;
  float s = 0.f;
  for (int b = rg; b < nblk; b += 8) s += slab[((long long)b * SCO + co) * SK + k];
  sh[rg][k] = s;
  __syncthreads();
  if (threadIdx.x < 27) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) t += sh[r][k];
    const int tap = k / 3, c = k - 3 * tap;
    float* d = dw + (co * 3 + c) * 9 + tap;
    *d = accumulate ? *d + t : t;
  }
}

// Merge per-block (n, mean, M2) rows [nblk][3][C] into the BN batch statistics
// (Chan et al.; double), then the same outputs as bn_stats_finalize (norm.hip).  ROW = true:
// write the merged (n, mean, M2) row [3][C] to save_mean instead (dg_bn_part_row).
template <bool ROW = false>
__global__ __launch_bounds__(SNT) void bn_part_finalize(const float* __restrict__ part, int nblk, int C,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float* running_mean,
                                                        float* running_var, float momentum, float eps,
                                                        float* save_mean, float* save_invstd, float* scale,
                                                        float* shift) {
  __shared__ double sh[2][SNT];
  __shared__ double smean;
  const int c = blockIdx.x, tid = threadIdx.x;
  const long long row = 3LL * C;
  double n = 0.0, s = 0.0;
  for (int b = tid; b < nblk; b += SNT) {
    const double nb = part[b * row + c];
    n += nb;
    s += nb * part[b * row + C + c];
  }
  sh[0][tid] = n; sh[1][tid] = s;
  __syncthreads();
  for (int o = SNT / 2; o > 0; o >>= 1) {
    if (tid < o) { sh[0][tid] += sh[0][tid + o]; sh[1][tid] += sh[1][tid + o]; }
    __syncthreads();
  }
  const double M = sh[0][0];
  if (tid == 0) smean = sh[1][0] / M;
  __syncthreads();
  const double mean = smean;
  double m2 = 0.0;
  for (int b = tid; b < nblk; b += SNT) {
    const double nb = part[b * row + c];
    if (nb == 0.0) continue;
    const double d = part[b * row + C + c] - mean;
    m2 += part[b * row + 2 * C + c] + nb * d * d;
  }
  __syncthreads();
  sh[0][tid] = m2;
  __syncthreads();
  for (int o = SNT / 2; o > 0; o >>= 1) {
    if (tid < o) sh[0][tid] += sh[0][tid + o];
    __syncthreads();
  }
  if (tid != 0) return;
  if constexpr (ROW) {
    save_mean[c] = (float)M;
    save_mean[C + c] = (float)mean;
    save_mean[2 * C + c] = (float)sh[0][0];
    return;
  }
  const double var = sh[0][0] / M;
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

// First stage of the partial merge for long partial lists: rows [64b, 64b+64) of
// part[nblk][3][C] -> out row b (Chan, float), 64 channels x 4 row groups per block.
constexpr int PMG = 64;
__global__ __launch_bounds__(SNT) void bn_part_merge(const float* __restrict__ part, int nblk, int C,
                                                     float* __restrict__ out) {
  __shared__ float sh[3][4][64];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const long long row = 3LL * C;
  const int r0 = blockIdx.y * PMG, r1 = min(nblk, r0 + PMG);
  float n = 0.f, mean = 0.f, m2 = 0.f;
  if (c < C) {
    // all of this thread's rows loaded up front (the Chan chain below is serial; loads issued
    // inside it waited one memory latency per row), merged in row order as before
    constexpr int RPT = PMG / 4;
    float nbv[RPT], mbv[RPT], m2v[RPT];
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const int b = r0 + rg + 4 * u;
      const bool in = b < r1;
      nbv[u] = in ? part[b * row + c] : 0.f;
      mbv[u] = in ? part[b * row + C + c] : 0.f;
      m2v[u] = in ? part[b * row + 2 * C + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
      const float nb = nbv[u];
      if (nb == 0.f) continue;
      const float nt = n + nb;
      const float d = mbv[u] - mean;
      mean += d * (nb / nt);
      m2 += m2v[u] + d * d * (n * nb / nt);
      n = nt;
    }
  }
  sh[0][rg][cl] = n; sh[1][rg][cl] = mean; sh[2][rg][cl] = m2;
  __syncthreads();
  if (rg != 0 || c >= C) return;
  n = 0.f; mean = 0.f; m2 = 0.f;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float nb = sh[0][g][cl];
    if (nb == 0.f) continue;
    const float nt = n + nb;
    const float d = sh[1][g][cl] - mean;
    mean += d * (nb / nt);
    m2 += sh[2][g][cl] + d * d * (n * nb / nt);
    n = nt;
  }
  float* o = out + (long long)blockIdx.y * row;
  o[c] = n; o[C + c] = mean; o[2 * C + c] = m2;
}

inline int part_rows2(int nblk) { return nblk > 1024 ? dg_cdiv(nblk, PMG) : 0; }

inline int stem_fwd_grid(long long nseg) { return (int)std::max(1LL, std::min(512LL, (nseg + 3) / 4)); }
// the apply pass (MODE 2) writes no statistics rows, so its grid is free of the 512-row layout:
// at 114 VGPRs four 256-thread blocks fit per CU (4 waves per SIMD instead of 2), which a
// streaming pass with one 1-KB store per pixel group needs to keep enough bytes in flight
// (DGVCC_STEM_APPLY_BPC = blocks per CU, default 4; 2 restores the statistics passes' grid)
inline int stem_apply_grid(long long nseg) {
  const char* e = getenv("DGVCC_STEM_APPLY_BPC");
  const long long bpc = e ? std::max(1, atoi(e)) : 4;
  return (int)std::max(1LL, std::min(256LL * bpc, (nseg + 3) / 4));
}
inline int stem_bwd_grid(long long nseg) { return (int)std::max(1LL, std::min(512LL, (nseg + 3) / 4)); }
constexpr int STEM_RPB = 32;  // slab rows per first-stage reduce block

}  // namespace

extern "C" int64_t dg_stem_part_rows(int N, int H, int W) {
  if (N <= 0 || H <= 0 || W <= 0) return DG_ERR_INVALID;
  return stem_fwd_grid((long long)N * H * (W / 64));
}

extern "C" int dg_stem_fwd(const float* img, int N, int H, int W, const void* wpack, const float* bias, void* z,
                           int64_t ldz, float* part, void* stream) {
  DG_REQUIRE(img && wpack && z && part && N > 0 && H > 0 && W > 0 && ldz >= SCO);
  DG_SUPPORTED(W % 64 == 0 && (long long)N * 3 * H * W < (1LL << 31) && ldz % 8 == 0);
  const long long nseg = (long long)N * H * (W / 64);
  hipLaunchKernelGGL(stem_fwd_kernel<0>, dim3(stem_fwd_grid(nseg)), dim3(SNT), 0, (hipStream_t)stream, img, H, W,
                     (const bf16*)wpack, bias, (bf16*)z, (long long)ldz, nseg, part, StemBn{});
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// fp32: wk = the filter as [k = (c*3 + r)*3 + s][64] f32, z f32 NHWC (same part rows).
extern "C" int dg_stem_fwd_f32(const float* img, int N, int H, int W, const float* wk, const float* bias, float* z,
                               int64_t ldz, float* part, void* stream) {
  DG_REQUIRE(img && wk && z && part && N > 0 && H > 0 && W > 0 && ldz >= SCO);
  DG_SUPPORTED(W % 64 == 0 && (long long)N * 3 * H * W < (1LL << 31) && ldz % 4 == 0);
  const long long nseg = (long long)N * H * (W / 64);
  hipLaunchKernelGGL(stem_fwd_f32_kernel, dim3(stem_fwd_grid(nseg)), dim3(SNT), 0, (hipStream_t)stream, img, H, W,
                     wk, bias, z, (long long)ldz, nseg, part);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// Statistics only (z not stored; its consumers recompute it from the image).
extern "C" int dg_stem_stats(const float* img, int N, int H, int W, const void* wpack, const float* bias, float* part,
                             void* stream) {
  DG_REQUIRE(img && wpack && part && N > 0 && H > 0 && W > 0);
  DG_SUPPORTED(W % 64 == 0 && (long long)N * 3 * H * W < (1LL << 31));
  const long long nseg = (long long)N * H * (W / 64);
  hipLaunchKernelGGL(stem_fwd_kernel<1>, dim3(stem_fwd_grid(nseg)), dim3(SNT), 0, (hipStream_t)stream, img, H, W,
                     (const bf16*)wpack, bias, (bf16*)nullptr, 0LL, nseg, part, StemBn{});
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// y = relu(scale * z + shift) with z = conv(img) + bias recomputed (bit-identical to
// dg_stem_fwd + dg_bn_apply on the stored z).
extern "C" int dg_stem_apply(const float* img, int N, int H, int W, const void* wpack, const float* bias,
                             const float* scale, const float* shift, void* y, int64_t ldy, void* stream) {
  DG_REQUIRE(img && wpack && scale && shift && y && N > 0 && H > 0 && W > 0 && ldy >= SCO);
  DG_SUPPORTED(W % 64 == 0 && (long long)N * 3 * H * W < (1LL << 31) && ldy % 8 == 0);
  const long long nseg = (long long)N * H * (W / 64);
  StemBn bn{scale, shift, nullptr, nullptr, nullptr, 0};
  hipLaunchKernelGGL(stem_fwd_kernel<2>, dim3(stem_apply_grid(nseg)), dim3(SNT), 0, (hipStream_t)stream, img, H, W,
                     (const bf16*)wpack, bias, (bf16*)y, (long long)ldy, nseg, (float*)nullptr, bn);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// BN-backward partial sums of the stem (z recomputed): part[dg_stem_part_rows][3][64] of
// (sum g', sum g' xhat, sum xhat), g' = g * relu'(scale z + shift); then bn_bwd_finalize.
extern "C" int dg_stem_bwd_coef(const float* img, int N, int H, int W, const void* wpack, const float* bias,
                                const void* g, int64_t ldg, const float* gamma, const float* save_mean,
                                const float* save_invstd, const float* scale, const float* shift, float* coef,
                                float* dgamma, float* dbeta, float* dbias, float* part, void* stream) {
  DG_REQUIRE(img && wpack && g && save_mean && save_invstd && scale && shift && coef && part && N > 0 && H > 0 &&
             W > 0 && ldg >= SCO);
  DG_SUPPORTED(W % 64 == 0 && (long long)N * 3 * H * W < (1LL << 31) && ldg % 8 == 0);
  const long long nseg = (long long)N * H * (W / 64);
  const int grid = stem_fwd_grid(nseg);
  StemBn bn{scale, shift, save_mean, save_invstd, (const bf16*)g, (long long)ldg};
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(stem_fwd_kernel<3>, dim3(grid), dim3(SNT), 0, st, img, H, W, (const bf16*)wpack, bias,
                     (bf16*)nullptr, 0LL, nseg, part, bn);
  DG_CHECK_LAUNCH();
  return dg_bn_bwd_finalize_part(part, grid, (int)(N * (long long)H * W), SCO, gamma, save_invstd, dgamma, dbeta,
                                 dbias, coef, stream);
}

extern "C" int64_t dg_bn_part_workspace(int nblk, int C) {
  if (nblk <= 0 || C <= 0) return DG_ERR_INVALID;
  return std::max<int64_t>(16, (int64_t)part_rows2(nblk) * 3 * C * 4);
}

extern "C" int dg_bn_part_finalize(const float* part, int nblk, int C, const float* gamma, const float* beta,
                                   float* running_mean, float* running_var, float momentum, float eps,
                                   float* save_mean, float* save_invstd, float* scale, float* shift, void* workspace,
                                   void* stream) {
  DG_REQUIRE(part && nblk > 0 && C > 0 && save_mean && save_invstd && scale && shift);
  DG_REQUIRE((running_mean == nullptr) == (running_var == nullptr));
  hipStream_t st = (hipStream_t)stream;
  const int r2 = part_rows2(nblk);
  if (r2) {  // long list: merge groups of 64 rows first
    DG_REQUIRE(workspace);
    hipLaunchKernelGGL(bn_part_merge, dim3(dg_cdiv(C, 64), r2), dim3(SNT), 0, st, part, nblk, C, (float*)workspace);
    DG_CHECK_LAUNCH();
    part = (const float*)workspace;
    nblk = r2;
  }
  hipLaunchKernelGGL(bn_part_finalize<false>, dim3(C), dim3(SNT), 0, st, part, nblk, C, gamma, beta, running_mean,
                     running_var, momentum, eps, save_mean, save_invstd, scale, shift);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

// The merged (n, mean, M2) row [3][C] of part[nblk][3][C]: one SyncBatchNorm rank's statistics,
// all-gathered and then finalized across ranks by dg_bn_part_finalize (nblk = world size).
extern "C" int dg_bn_part_row(const float* part, int nblk, int C, float* row, void* workspace, void* stream) {
  DG_REQUIRE(part && row && nblk > 0 && C > 0);
  hipStream_t st = (hipStream_t)stream;
  const int r2 = part_rows2(nblk);
  if (r2) {
    DG_REQUIRE(workspace);
    hipLaunchKernelGGL(bn_part_merge, dim3(dg_cdiv(C, 64), r2), dim3(SNT), 0, st, part, nblk, C, (float*)workspace);
    DG_CHECK_LAUNCH();
    part = (const float*)workspace;
    nblk = r2;
  }
  hipLaunchKernelGGL(bn_part_finalize<true>, dim3(C), dim3(SNT), 0, st, part, nblk, C, nullptr, nullptr, nullptr,
                     nullptr, 0.f, 0.f, row, nullptr, nullptr, nullptr);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int64_t dg_stem_bwd_workspace(int N, int H, int W) {
  if (N <= 0 || H <= 0 || W <= 0) return DG_ERR_INVALID;
  const int grid = stem_bwd_grid((long long)N * H * (W / 32));
  return ((int64_t)grid + dg_cdiv(grid, STEM_RPB)) * SCO * SK * 4;
}

// z == NULL: z is recomputed from img with the packed filters wpack (+ bias), as dg_stem_stats
// / dg_stem_apply do, instead of read from HBM.
// fp32: g, z f32 (pixel strides ldg, ldz % 4 == 0); same workspace, reduction and dw layout.
extern "C" int dg_stem_bwd_f32(const float* img, int N, int H, int W, const float* g, int64_t ldg, const float* z,
                               int64_t ldz, const float* save_mean, const float* save_invstd, const float* scale,
                               const float* shift, const float* coef, float* dw, void* workspace, int64_t ws_bytes,
                               int accumulate, void* stream) {
  DG_REQUIRE(img && g && z && save_mean && save_invstd && scale && shift && coef && dw && workspace);
  DG_REQUIRE(N > 0 && H > 0 && W > 0 && ldg >= SCO && ldz >= SCO);
  DG_SUPPORTED(W % 32 == 0 && (long long)N * 3 * H * W < (1LL << 31) && ldg % 4 == 0 && ldz % 4 == 0);
  const long long nseg = (long long)N * H * (W / 32);
  const int grid = stem_bwd_grid(nseg);
  const int nred = dg_cdiv(grid, STEM_RPB);
  DG_REQUIRE(ws_bytes >= ((int64_t)grid + nred) * SCO * SK * 4);
  hipStream_t st = (hipStream_t)stream;
  float* slab = (float*)workspace;
  float* slab2 = slab + (long long)grid * SCO * SK;
  hipLaunchKernelGGL(stem_bwd_f32_kernel, dim3(grid), dim3(SNT), 0, st, img, H, W, g, (long long)ldg, z,
                     (long long)ldz, save_mean, save_invstd, scale, shift, coef, nseg, slab);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(colsum_rows_kernel, dim3(SCO * SK / SNT, nred), dim3(SNT), 0, st, (const float*)slab, grid,
                     SCO * SK, STEM_RPB, slab2);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(stem_wgrad_reduce, dim3(SCO), dim3(SNT), 0, st, (const float*)slab2, nred, dw, accumulate);
  DG_CHECK_LAUNCH();
  return DG_OK;
}

extern "C" int dg_stem_bwd(const float* img, int N, int H, int W, const void* g, int64_t ldg, const void* z,
                           int64_t ldz, const float* save_mean, const float* save_invstd, const float* scale,
                           const float* shift, const float* coef, float* dw, void* workspace, int64_t ws_bytes,
                           int accumulate, const void* wpack, const float* bias, void* stream) {
  DG_REQUIRE(img && g && save_mean && save_invstd && scale && shift && coef && dw && workspace && (z || wpack));
  DG_REQUIRE(N > 0 && H > 0 && W > 0 && ldg >= SCO && (!z || ldz >= SCO));
  DG_SUPPORTED(W % 32 == 0 && (long long)N * 3 * H * W < (1LL << 31) && ldg % 8 == 0 && (!z || ldz % 8 == 0));
  const long long nseg = (long long)N * H * (W / 32);
  const int grid = stem_bwd_grid(nseg);
  const int nred = dg_cdiv(grid, STEM_RPB);
  DG_REQUIRE(ws_bytes >= ((int64_t)grid + nred) * SCO * SK * 4);
  hipStream_t st = (hipStream_t)stream;
  float* slab = (float*)workspace;
  float* slab2 = slab + (long long)grid * SCO * SK;
  if (z)
    hipLaunchKernelGGL(stem_bwd_kernel<0>, dim3(grid), dim3(SNT), 0, st, img, H, W, (const bf16*)g, (long long)ldg,
                       (const bf16*)z, (long long)ldz, save_mean, save_invstd, scale, shift, coef, nseg, slab,
                       (const bf16*)nullptr, (const float*)nullptr);
  else
    hipLaunchKernelGGL(stem_bwd_kernel<1>, dim3(grid), dim3(SNT), 0, st, img, H, W, (const bf16*)g, (long long)ldg,
                       (const bf16*)nullptr, 0LL, save_mean, save_invstd, scale, shift, coef, nseg, slab,
                       (const bf16*)wpack, bias);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(colsum_rows_kernel, dim3(SCO * SK / SNT, nred), dim3(SNT), 0, st, (const float*)slab, grid,
                     SCO * SK, STEM_RPB, slab2);
  DG_CHECK_LAUNCH();
  hipLaunchKernelGGL(stem_wgrad_reduce, dim3(SCO), dim3(SNT), 0, st, (const float*)slab2, nred, dw, accumulate);
  DG_CHECK_LAUNCH();
  return DG_OK;
}
