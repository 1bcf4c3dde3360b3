// Single-token decode attention over a KV cache (gfx950), for KV-cached greedy generation.
//
// The reference decodes by re-running the whole prefix for every token (test.py:144-150).
// generation.py keeps per-layer (B, T_max, H_local, hd) key / value caches instead; every
// decode step appends one key/value row per sequence and attends one query row per
// (sequence, head) against all cached keys.  That is a memory-bound GEMV-shaped problem
// (a few MB of cache per layer, no MFMA-sized tiles), so the kernels here are VALU/LDS
// split-K ("flash-decoding"):
//
//   attn_decode_split_k  grid (T_max/256 splits, B*H): one workgroup scores 256 keys, 4 waves
//                        x 64 keys, lane-per-key dot products (q held in registers), wave
//                        softmax, then P.V with lanes = 8 key groups x 8 dim groups (16-byte V
//                        loads) and an xor-shuffle reduction; the 4 waves merge through LDS
//                        into one (max, sum, o[hd]) fp32 partial per split.
//   attn_decode_combine_k one wave per (b, h) merges the partials of the live splits.
//
// The current length is read from DEVICE memory (len_ptr), never from a kernel argument, and
// the grid covers T_max: the whole decode step can be captured once in a HIP graph and
// replayed for every token (splits past the length exit at once).  kv_append_k writes the
// new token's (RoPE-rotated) key / value rows at row *len_ptr; step_advance_k bumps the
// length and the position ids on the device at the end of the step.
#include "common.h"

namespace dpfs {

constexpr int kSplit = 256;   // keys per workgroup

template <int HD>
__global__ __launch_bounds__(256) void attn_decode_split_k(const bf16* __restrict__ q, long long ldq,
                                                          const bf16* __restrict__ kc, const bf16* __restrict__ vc,
                                                          const int* __restrict__ len_ptr, int H, int Tmax,
                                                          float scale, float* __restrict__ part) {
  constexpr int NV = HD / 8;               // 16-byte vectors per row
  const int split = blockIdx.x, bh = blockIdx.y, b = bh / H, h = bh % H;
  const int L = min(*len_ptr + 1, Tmax);  // cached keys + the token being decoded
  const int k0 = split * kSplit;
  float* out = part + ((long long)bh * gridDim.x + split) * (HD + 2);
  if (k0 >= L) return;                     // the combine kernel never reads this split
  const int wave = threadIdx.x >> 6, l = lane_id();
  __shared__ float p_lds[4][64];
  __shared__ float o_lds[4][HD];
  __shared__ float ml_lds[4][2];

  // q in registers (every lane holds the full row for its own key's dot product)
  float qf[HD];
  const bf16* qrow = q + (long long)b * ldq + (long long)h * HD;
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    float v[8];
    load_vec<bf16>(qrow + 8 * c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[8 * c + j] = v[j] * scale;
  }
  // scores: lane-per-key
  const int key = k0 + wave * 64 + l;
  float s = -INFINITY;
  if (key < L) {
    const bf16* krow = kc + (((long long)b * Tmax + key) * H + h) * HD;
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      float v[8];
      load_vec<bf16>(krow + 8 * c, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc = fmaf(qf[8 * c + j], v[j], acc);
    }
    s = acc;
  }
  const float m = wave_max(s);
  float p = (key < L && m != -INFINITY) ? __expf(s - m) : 0.f;
  const float lsum = wave_sum(p);
  p_lds[wave][l] = p;
  __syncthreads();
  // P.V: lane = (key group kg, dim group dg) with DG dim groups of DPL dims (16-byte V
  // loads); each lane walks DG keys of the wave's 64, then the KG key groups are summed.
  constexpr int DG = HD >= 64 ? 8 : HD / 8;   // dim groups: 8 at hd 64 / 128, 4 at hd 32
  constexpr int DPL = HD / DG;                // dims per lane: 8 (hd 32 / 64) or 16 (hd 128)
  constexpr int KG = 64 / DG;                 // key groups
  const int kg = l / DG, dg = l % DG;
  float o[DPL];
#pragma unroll
  for (int j = 0; j < DPL; ++j) o[j] = 0.f;
  const int kw0 = k0 + wave * 64;
#pragma unroll
  for (int i = 0; i < DG; ++i) {
    const int kk = kg + KG * i;             // key within the wave's 64
    const float pk = p_lds[wave][kk];
    if (kw0 + kk < L) {
      const bf16* vrow = vc + (((long long)b * Tmax + kw0 + kk) * H + h) * HD + dg * DPL;
#pragma unroll
      for (int c = 0; c < DPL / 8; ++c) {
        float v[8];
        load_vec<bf16>(vrow + 8 * c, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[8 * c + j] = fmaf(pk, v[j], o[8 * c + j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < DPL; ++j) {          // sum over the key groups (lanes l ^ DG, 2 DG, ...)
    float v = o[j];
#pragma unroll
    for (int x = DG; x < 64; x <<= 1) v += __shfl_xor(v, x, 64);
    o[j] = v;
  }
  if (kg == 0) {
#pragma unroll
    for (int j = 0; j < DPL; ++j) o_lds[wave][dg * DPL + j] = o[j];
  }
  if (l == 0) {
    ml_lds[wave][0] = m;
    ml_lds[wave][1] = lsum;
  }
  __syncthreads();
  // merge the 4 waves (fixed order) into this split's partial
  if (threadIdx.x < HD) {
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, ml_lds[w][0]);
    float acc = 0.f, ls = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float mw = ml_lds[w][0];
      const float f = mw == -INFINITY ? 0.f : __expf(mw - M);
      acc += f * o_lds[w][threadIdx.x];
      ls += f * ml_lds[w][1];
    }
    out[2 + threadIdx.x] = acc;
    if (threadIdx.x == 0) {
      out[0] = M;
      out[1] = ls;
    }
  }
}

template <int HD>
__global__ __launch_bounds__(64) void attn_decode_combine_k(const float* __restrict__ part, int nsplit,
                                                           const int* __restrict__ len_ptr, bf16* __restrict__ o,
                                                           long long ldo, int H) {
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int L = min(*len_ptr + 1, nsplit * kSplit);
  const int live = (L + kSplit - 1) / kSplit;
  const float* p = part + (long long)bh * nsplit * (HD + 2);
  float M = -INFINITY;
  for (int s = 0; s < live; ++s) M = fmaxf(M, p[s * (HD + 2)]);
  constexpr int DPL = HD >= 64 ? HD / 64 : 1;   // hd 32: lanes >= 32 idle
  const bool on = (int)threadIdx.x < HD;
  float acc[DPL];
#pragma unroll
  for (int j = 0; j < DPL; ++j) acc[j] = 0.f;
  float ls = 0.f;
  for (int s = 0; s < live; ++s) {
    const float* ps = p + s * (HD + 2);
    const float f = __expf(ps[0] - M);
    ls += f * ps[1];
#pragma unroll
    for (int j = 0; j < DPL; ++j)
      if (on) acc[j] += f * ps[2 + threadIdx.x + 64 * j];
  }
  const float inv = 1.f / ls;
  bf16* orow = o + (long long)b * ldo + (long long)h * HD;
#pragma unroll
  for (int j = 0; j < DPL; ++j)
    if (on) orow[threadIdx.x + 64 * j] = (bf16)(acc[j] * inv);
}

// cache[b, *len, h, :] = src rows (k and v parts of the packed qkv row of sequence b)
__global__ __launch_bounds__(256) void kv_append_k(const bf16* __restrict__ ksrc, const bf16* __restrict__ vsrc,
                                                  long long ld, bf16* __restrict__ kc, bf16* __restrict__ vc,
                                                  const int* __restrict__ len_ptr, int B, int H, int HD, int Tmax) {
  const int t = *len_ptr;
  if (t < 0 || t >= Tmax) return;          // full cache: nothing to append (never out of bounds)
  const int nv = H * HD / 8;               // 16-byte vectors per token row
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 2 * B * nv; i += gridDim.x * blockDim.x) {
    const int isv = i >= B * nv;
    const int j = isv ? i - B * nv : i;
    const int b = j / nv, c = j % nv;
    const bf16* src = (isv ? vsrc : ksrc) + (long long)b * ld + 8 * c;
    bf16* dst = (isv ? vc : kc) + ((long long)b * Tmax + t) * H * HD + 8 * c;
    *reinterpret_cast<u32x4*>(dst) = *reinterpret_cast<const u32x4*>(src);
  }
}

// -------------------------------------------------------------- small-M projections --
// y[M, N] (+ bias) = A[M, K] W[N, K]^T for M <= 16 rows (the decode step's projections: one
// row per sequence).  hipBLASLt's tiles for these shapes move ~0.5 TB/s of W (7 us for the
// 3.5 MB GPT-2 QKV weight); here each wave is one v_mfma_f32_16x16x32_bf16 chain: the M rows
// are its A tile (rows >= M read as zeros), 16 rows of W its B tile (4 lanes x 16 B per row
// segment), and the KS waves of a workgroup split K and merge in LDS in a fixed order.  W is
// streamed once with all of a wave's loads issued ahead of its MFMAs; A (a few KB) stays in
// L2.  SW: A = silu(g) * u of a packed [M, 2K] gate|up input -- the SwiGLU fused into the down
// projection's operand load (same fp32 formula and bf16 rounding as swiglu_fwd_k).
__device__ __forceinline__ float silu_dec(float g) { return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)); }   // = silu_f

template <int KS, bool SW>
__global__ __launch_bounds__(64 * KS) void gemv16_k(const bf16* __restrict__ A, long long lda,
                                                    const bf16* __restrict__ W, long long ldw,
                                                    const float* __restrict__ bias, bf16* __restrict__ Y,
                                                    long long ldy, int M, int N, int K) {
  constexpr int CH = 8;                      // MFMA k-steps per batch of loads
  __shared__ f32x4 red[KS][64];
  const int wave = threadIdx.x >> 6, l = lane_id(), g = l >> 4, i = l & 15;
  const int n0 = blockIdx.x * 16;
  const int nk = K / 32;
  const int per = (nk + KS - 1) / KS;
  const int c0 = wave * per, c1 = min(nk, c0 + per);
  const bf16* wp = W + (long long)min(n0 + i, N - 1) * ldw + 8 * g;
  const bool mv = i < M;
  const bf16* ap = A + (long long)(mv ? i : 0) * lda + 8 * g;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int cb = c0; cb < c1; cb += CH) {
    bf16x8 b[CH], a[CH];
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int c = cb + u;
      if (c < c1) {
        b[u] = *reinterpret_cast<const bf16x8*>(wp + 32 * c);
        if (SW) {
          const bf16x8 gv = *reinterpret_cast<const bf16x8*>(ap + 32 * c);
          const bf16x8 uv = *reinterpret_cast<const bf16x8*>(ap + K + 32 * c);
#pragma unroll
          for (int j = 0; j < 8; ++j) a[u][j] = (bf16)(silu_dec((float)gv[j]) * (float)uv[j]);
        } else {
          a[u] = *reinterpret_cast<const bf16x8*>(ap + 32 * c);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      if (cb + u < c1) {
        const bf16x8 z = {};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(mv ? a[u] : z, b[u], acc, 0, 0, 0);
      }
    }
  }
  red[wave][l] = acc;
  __syncthreads();
  if (wave == 0) {
#pragma unroll
    for (int w = 1; w < KS; ++w) acc += red[w][l];
    const int n = n0 + i;                    // D[row = 4g + j][col = lane & 15]
    if (n < N) {
      const float bv = bias ? bias[n] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = 4 * g + j;
        if (m < M) Y[(long long)m * ldy + n] = (bf16)(acc[j] + bv);
      }
    }
  }
}

// RoPE of the q and k heads of the packed qkv rows (in place) fused with the cache append of
// the rotated k row and the v row at row *len: one launch instead of rope_k + kv_append_k.
// Same arithmetic and rounding as rope_vec_k (sign +1).  8 frequency pairs per thread.
__global__ __launch_bounds__(256) void rope_append_k(bf16* __restrict__ qkv, long long ld,
                                                     const int64_t* __restrict__ pos,
                                                     const float* __restrict__ tab, bf16* __restrict__ kc,
                                                     bf16* __restrict__ vc, const int* __restrict__ len_ptr,
                                                     int B, int H, int HD, int Tmax) {
  const int t = *len_ptr;
  const bool app = t >= 0 && t < Tmax;     // full cache: rotate, append nothing
  const int h2 = HD / 2, q8 = h2 / 8;
  const int rot_per_b = 2 * H * q8;
  const int nrot = B * rot_per_b;
  const int vpr = H * HD / 8;              // 16-byte v vectors per sequence
  const int total = nrot + B * vpr;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    if (i < nrot) {
      const int b = i / rot_per_b, r = i - b * rot_per_b;
      const int head = r / q8, f0 = (r - head * q8) * 8;
      bf16* base = qkv + (long long)b * ld + head * HD;
      KASSERT(pos[b] >= 0, "decode position %lld of sequence %d", (long long)pos[b], b);
      const float* tr = tab + pos[b] * (long long)HD;
      const bf16x8 xa = *reinterpret_cast<const bf16x8*>(base + f0);
      const bf16x8 xb = *reinterpret_cast<const bf16x8*>(base + h2 + f0);
      bf16x8 oa, ob;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float c = tr[f0 + j], sn = tr[h2 + f0 + j];
        const float x1 = (float)xa[j], x2 = (float)xb[j];
        oa[j] = (bf16)(x1 * c - x2 * sn);
        ob[j] = (bf16)(x2 * c + x1 * sn);
      }
      *reinterpret_cast<bf16x8*>(base + f0) = oa;
      *reinterpret_cast<bf16x8*>(base + h2 + f0) = ob;
      if (head >= H && app) {
        bf16* dst = kc + (((long long)b * Tmax + t) * H + (head - H)) * HD;
        *reinterpret_cast<bf16x8*>(dst + f0) = oa;
        *reinterpret_cast<bf16x8*>(dst + h2 + f0) = ob;
      }
    } else if (app) {
      const int j = i - nrot, b = j / vpr, c = j - b * vpr;
      const bf16* src = qkv + (long long)b * ld + 2 * H * HD + 8 * c;
      bf16* dst = vc + ((long long)b * Tmax + t) * H * HD + 8 * c;
      *reinterpret_cast<u32x4*>(dst) = *reinterpret_cast<const u32x4*>(src);
    }
  }
}

// *len += 1; pos[b] = *len (the next token's position) for every sequence.
__global__ void step_advance_k(int* __restrict__ len_ptr, int64_t* __restrict__ pos, int B) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const int t = *len_ptr + 1;
    *len_ptr = t;
    for (int b = 0; b < B; ++b) pos[b] = t;
  }
}

}  // namespace dpfs

using namespace dpfs;

extern "C" int dpfs_decode_nsplit(int Tmax) { return (Tmax + kSplit - 1) / kSplit; }

extern "C" void dpfs_attn_decode(const void* q, long long ldq, const void* kc, const void* vc, const int* len_ptr,
                                 void* o, long long ldo, float* part, int B, int H, int HD, int Tmax, float scale,
                                 hipStream_t s) {
  const int ns = dpfs_decode_nsplit(Tmax);
  const dim3 grid(ns, B * H);
  if (HD == 32) {
    attn_decode_split_k<32><<<grid, 256, 0, s>>>((const bf16*)q, ldq, (const bf16*)kc, (const bf16*)vc, len_ptr, H,
                                                  Tmax, scale, part);
    attn_decode_combine_k<32><<<B * H, 64, 0, s>>>(part, ns, len_ptr, (bf16*)o, ldo, H);
  } else if (HD == 64) {
    attn_decode_split_k<64><<<grid, 256, 0, s>>>((const bf16*)q, ldq, (const bf16*)kc, (const bf16*)vc, len_ptr, H,
                                                  Tmax, scale, part);
    attn_decode_combine_k<64><<<B * H, 64, 0, s>>>(part, ns, len_ptr, (bf16*)o, ldo, H);
  } else {
    attn_decode_split_k<128><<<grid, 256, 0, s>>>((const bf16*)q, ldq, (const bf16*)kc, (const bf16*)vc, len_ptr, H,
                                                   Tmax, scale, part);
    attn_decode_combine_k<128><<<B * H, 64, 0, s>>>(part, ns, len_ptr, (bf16*)o, ldo, H);
  }
}

extern "C" void dpfs_kv_append(const void* ksrc, const void* vsrc, long long ld, void* kc, void* vc,
                               const int* len_ptr, int B, int H, int HD, int Tmax, hipStream_t s) {
  const int n = 2 * B * H * HD / 8;
  kv_append_k<<<(n + 255) / 256, 256, 0, s>>>((const bf16*)ksrc, (const bf16*)vsrc, ld, (bf16*)kc, (bf16*)vc,
                                              len_ptr, B, H, HD, Tmax);
}

extern "C" void dpfs_step_advance(int* len_ptr, int64_t* pos, int B, hipStream_t s) {
  step_advance_k<<<1, 64, 0, s>>>(len_ptr, pos, B);
}

extern "C" int dpfs_gemv16_ok(int M, int N, int K, long long lda, long long ldw) {
  return M >= 1 && M <= 16 && N >= 1 && K % 32 == 0 && K > 0 && lda % 8 == 0 && ldw % 8 == 0;
}

extern "C" void dpfs_gemv16(const void* A, long long lda, const void* W, long long ldw, const float* bias, void* Y,
                            long long ldy, int M, int N, int K, int swiglu, hipStream_t s) {
  const int nb = (N + 15) / 16;
  // K split over 8 waves while that still leaves >= 2 MFMA k-steps per wave and the grid is
  // small; 4 waves for wide N (the lm_head: thousands of workgroups already)
  const bool ks8 = nb <= 512 && K / 32 >= 16;
  if (ks8) {
    if (swiglu) gemv16_k<8, true><<<nb, 512, 0, s>>>((const bf16*)A, lda, (const bf16*)W, ldw, bias, (bf16*)Y, ldy, M, N, K);
    else gemv16_k<8, false><<<nb, 512, 0, s>>>((const bf16*)A, lda, (const bf16*)W, ldw, bias, (bf16*)Y, ldy, M, N, K);
  } else {
    if (swiglu) gemv16_k<4, true><<<nb, 256, 0, s>>>((const bf16*)A, lda, (const bf16*)W, ldw, bias, (bf16*)Y, ldy, M, N, K);
    else gemv16_k<4, false><<<nb, 256, 0, s>>>((const bf16*)A, lda, (const bf16*)W, ldw, bias, (bf16*)Y, ldy, M, N, K);
  }
}

extern "C" void dpfs_rope_append(void* qkv, long long ld, const int64_t* pos, const float* tab, void* kc, void* vc,
                                 const int* len_ptr, int B, int H, int HD, int Tmax, hipStream_t s) {
  const int total = B * 2 * H * (HD / 16) + B * H * HD / 8;
  const int grid = (total + 255) / 256;
  rope_append_k<<<grid, 256, 0, s>>>((bf16*)qkv, ld, pos, tab, (bf16*)kc, (bf16*)vc, len_ptr, B, H, HD, Tmax);
}
