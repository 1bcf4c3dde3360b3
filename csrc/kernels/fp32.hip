// fp32 compute path on gfx950: the reference trains in fp32 unless --bf16 is passed
// (/root/reference/train.py:58-63), so that mode runs on these kernels instead of the PyTorch
// oracle.  gfx950 has no xf32: the fp32-input MFMAs (v_mfma_f32_32x32x2_f32) are exact fp32
// (an fmaf chain) at the vector rate, 1/16 of bf16 (MI355X_MICROARCH 'Matrix cores').
//
//  * gemm_f32_k<AK, BK>: C[M][N] (+)= op(A) op(B) (+ bias[N]) for the three layouts of a
//    parallel linear (NT forward, NN data gradient, TN weight gradient): 128 x 128 tiles,
//    four waves of 64 x 64 (2 x 2 MFMA tiles of 32 x 32), 16-deep K stages double-buffered
//    in LDS as [k][m] / [k][n] rows (so every MFMA operand is one conflict-free ds_read_b32
//    per lane: lane = row / column, k = lane >> 5), the next stage's global loads in flight
//    under the current stage's MFMAs.
//  * attn_fwd_f32_k / attn_bwd_dq_f32_k / attn_bwd_dkdv_f32_k: causal flash attention with the
//    bf16 kernels' orientation (attention.hip v3): forward and dQ compute S^T = K Q^T (query on
//    the lane, lane-local softmax), so P^T / dS^T in registers are directly the B operands of
//    O^T += V^T P^T and dQ^T += K^T dS^T -- MFMA step s = 4 g + j takes register s of each lane,
//    i.e. key 8 g + 4 (lane >> 5) + j, and the A operand is read for exactly that key; dK/dV
//    computes S = Q K^T with the key on the lane.  K / V / Q / dO tiles are fp32 in LDS with
//    a row stride of HD + 1 floats (conflict-free column reads).  Only the log-sum-exp is saved.
#include "common.h"

#include <algorithm>

namespace dpfs {

#define MFMA_F32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), 0, 0, 0)

// ------------------------------------------------------------------------------ GEMM --
constexpr int kF32BM = 128, kF32BK = 32, kF32LD = 128 + 4;   // LDS row: 128 floats + pad

// One 128 x 16 operand tile: AKM = true when the operand is K-major in memory (x[r][k], ld
// elements per row), false when it is MN-major (x[k][r]).  LDS image: s[k][r], fp32.  TI: the
// operand's storage (fp32, or bf16 for the GEMMs whose contiguous dimension the bf16 MFMA
// kernels cannot take: any alignment, converted to fp32 on the way in, exact products).
template <typename TI>
__device__ __forceinline__ f32x4 ld4(const TI* p) {
  if constexpr (sizeof(TI) == 4) {
    return *reinterpret_cast<const f32x4*>(p);
  } else {
    const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
    return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
  }
}
template <bool AKM, typename TI = float>
struct F32Tile {
  static constexpr int NI = kF32BK / 8;       // 16-byte pieces per thread (128 x BK floats / 256)
  static constexpr int TPR = kF32BK / 4;      // K-major: threads per row
  f32x4 v[NI];
  __device__ __forceinline__ void load(const TI* __restrict__ x, long long ld, int R, int Kd, int r0, int k0,
                                       bool vec) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      f32x4 q = {0.f, 0.f, 0.f, 0.f};
      if constexpr (AKM) {
        const int r = t / TPR + (256 / TPR) * i, k = (t % TPR) * 4;
        const int gr = r0 + r, gk = k0 + k;
        if (gr < R) {
          if (vec && gk + 3 < Kd) {
            q = ld4<TI>(x + (long long)gr * ld + gk);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) q[j] = gk + j < Kd ? to_f(x[(long long)gr * ld + gk + j]) : 0.f;
          }
        }
      } else {
        const int k = t / 32 + 8 * i, r = (t & 31) * 4;
        const int gr = r0 + r, gk = k0 + k;
        if (gk < Kd) {
          if (vec && gr + 3 < R) {
            q = ld4<TI>(x + (long long)gk * ld + gr);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) q[j] = gr + j < R ? to_f(x[(long long)gk * ld + gr + j]) : 0.f;
          }
        }
      }
      v[i] = q;
    }
  }
  __device__ __forceinline__ void store(float* s) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      if constexpr (AKM) {
        const int r = t / TPR + (256 / TPR) * i, k = (t % TPR) * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) s[(k + j) * kF32LD + r] = v[i][j];
      } else {
        const int k = t / 32 + 8 * i, r = (t & 31) * 4;
        *reinterpret_cast<f32x4*>(s + k * kF32LD + r) = v[i];
      }
    }
  }
};

// AK: A is K-major (a[m][k]); BK: B is K-major (b[n][k]).  C row-major fp32 with ldc.
// Split-K (blockIdx.y = split s of gridDim.y): the K range [s kps, min(K, (s + 1) kps)) into the
// fp32 slab C + s * slab (accumulate off); splitk_sum_f32_k adds the slabs in split order.
template <bool AK, bool BK, typename TI = float, typename TO = float>
__global__ __launch_bounds__(256) void gemm_f32_k(const TI* __restrict__ A, const TI* __restrict__ B,
                                                  TO* __restrict__ C, const float* __restrict__ bias, int M, int N,
                                                  int K, long long lda, long long ldb, long long ldc, int accumulate,
                                                  int vec_a, int vec_b, int kps, long long slab) {
  {
    const int kb = blockIdx.y * kps;
    const int ke = min(K, kb + kps);
    if (gridDim.y > 1) {   // this split's operand panels and output slab
      A += AK ? (long long)kb : (long long)kb * lda;
      B += BK ? (long long)kb : (long long)kb * ldb;
      C += blockIdx.y * slab;
      K = ke - kb;
    }
  }
  __shared__ __attribute__((aligned(16))) float sa[2][kF32BK * kF32LD];
  __shared__ __attribute__((aligned(16))) float sb[2][kF32BK * kF32LD];
  const int tiles_n = (N + kF32BM - 1) / kF32BM;
  const int tiles_m = (M + kF32BM - 1) / kF32BM;
  // XCD-aware order: consecutive ids share an XCD, and walk the tiles of one M panel
  const int id = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (id / tiles_n) * kF32BM, n0 = (id % tiles_n) * kF32BM;
  const int wave = threadIdx.x >> 6, l = lane_id(), r32 = l & 31, hf = l >> 5;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  F32Tile<AK, TI> ta;
  F32Tile<BK, TI> tb;
  const int nk = (K + kF32BK - 1) / kF32BK;
  ta.load(A, lda, M, K, m0, 0, vec_a);
  tb.load(B, ldb, N, K, n0, 0, vec_b);
  ta.store(sa[0]);
  tb.store(sb[0]);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {   // next stage's global loads fly under this stage's MFMAs
      ta.load(A, lda, M, K, m0, (kt + 1) * kF32BK, vec_a);
      tb.load(B, ldb, N, K, n0, (kt + 1) * kF32BK, vec_b);
    }
    const float* pa = sa[cur];
    const float* pb = sb[cur];
#pragma unroll
    for (int kk = 0; kk < kF32BK / 2; ++kk) {
      const int row = (2 * kk + hf) * kF32LD;
      const float a0 = pa[row + wm + r32], a1 = pa[row + wm + 32 + r32];
      const float b0 = pb[row + wn + r32], b1 = pb[row + wn + 32 + r32];
      acc[0][0] = MFMA_F32(a0, b0, acc[0][0]);
      acc[0][1] = MFMA_F32(a0, b1, acc[0][1]);
      acc[1][0] = MFMA_F32(a1, b0, acc[1][0]);
      acc[1][1] = MFMA_F32(a1, b1, acc[1][1]);
    }
    if (kt + 1 < nk) {
      ta.store(sa[cur ^ 1]);
      tb.store(sb[cur ^ 1]);
    }
    __syncthreads();
  }
  // epilogue: register r of tile (i, j) is row 8 (r >> 2) + 4 hf + (r & 3), column r32
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn + 32 * j + r32;
    if (col >= N) continue;
    const float bv = bias ? bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * i + 8 * (r >> 2) + 4 * hf + (r & 3);
        if (row < M) {
          TO* p = C + (long long)row * ldc + col;
          const float v = acc[i][j][r] + bv;
          *p = from_f<TO>(accumulate ? to_f(*p) + v : v);
        }
      }
  }
}

// ------------------------------------------------------------------------- attention --
// fp32 tiles in LDS: [rows][HD + 1] (the +1 keeps a 32-lane column read on 32 banks).
template <int HD>
struct F32Rows {
  static constexpr int LD = HD + 1;
  // the same tile in two halves: fetch = the global loads into registers (issued a tile ahead,
  // so their latency hides under the current tile's MFMAs -- these kernels run one or two waves
  // per SIMD, nothing else covers it), put = the LDS writes
  template <int R>
  struct Regs {
    static constexpr int N = (R * HD / 4 + 255) / 256;
    f32x4 v[N];
  };
  template <int R>
  __device__ __forceinline__ static void fetch(Regs<R>& g, const float* __restrict__ x, long long ld, int r0, int T) {
#pragma unroll
    for (int n = 0; n < Regs<R>::N; ++n) {
      const int i = threadIdx.x + 256 * n;
      const int r = i / (HD / 4), c = (i % (HD / 4)) * 4;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (i < R * HD / 4 && r0 + r < T) v = *reinterpret_cast<const f32x4*>(x + (long long)(r0 + r) * ld + c);
      g.v[n] = v;
    }
  }
  template <int R>
  __device__ __forceinline__ static void put(float* s, const Regs<R>& g) {
#pragma unroll
    for (int n = 0; n < Regs<R>::N; ++n) {
      const int i = threadIdx.x + 256 * n;
      const int r = i / (HD / 4), c = (i % (HD / 4)) * 4;
      if (i < R * HD / 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) s[r * LD + c + j] = g.v[n][j];
      }
    }
  }
  // rows [r0, r0 + R) of a (B, T, H, HD) view (row stride ld elements) into s; rows >= T zero
  template <int R>
  __device__ __forceinline__ static void load(float* s, const float* __restrict__ x, long long ld, int r0, int T) {
    for (int i = threadIdx.x; i < R * HD / 4; i += 256) {
      const int r = i / (HD / 4), c = (i % (HD / 4)) * 4;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (r0 + r < T) v = *reinterpret_cast<const f32x4*>(x + (long long)(r0 + r) * ld + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) s[r * LD + c + j] = v[j];
    }
  }
};

__device__ __forceinline__ float pair_max_f(float x) {
  return fmaxf(x, __shfl_xor(x, 32, 64));
}
__device__ __forceinline__ float pair_sum_f(float x) { return x + __shfl_xor(x, 32, 64); }

constexpr float kF32Log2e = 1.4426950408889634f;

// Forward: a workgroup = 4 waves x 32 queries of one (b, h); key tiles of 64 through LDS.
// S^T = K Q^T: A = K[key][d] (lane: key r32, d = 2 kk + hf), B = Q^T (lane: query r32, the
// same d: Q held in 2 registers per k-pair); O^T += V^T P^T with step s = 4 g + j reading
// V[8 g + 4 hf + j][d].
template <int HD>
__global__ __launch_bounds__(256) void attn_fwd_f32_k(const float* __restrict__ Q, const float* __restrict__ K,
                                                      const float* __restrict__ V, float* __restrict__ O,
                                                      float* __restrict__ LSE, int T, int H, long long ldq,
                                                      long long ldk, long long ldv, long long ldo, float scale,
                                                      int causal) {
  constexpr int BQ = 128, BKV = 64, KP = HD / 2, DT = HD / 32, LD = HD + 1;
  __shared__ float sk[BKV * LD], sv[BKV * LD];
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int qb = gridDim.x - 1 - blockIdx.x;   // heaviest (causal) blocks first
  const int q0 = qb * BQ, wave = threadIdx.x >> 6, l = lane_id(), r32 = l & 31, hf = l >> 5;
  const int qi = q0 + 32 * wave + r32;
  const float* qb_ = Q + (long long)b * T * ldq + (long long)h * HD;
  const float* kb_ = K + (long long)b * T * ldk + (long long)h * HD;
  const float* vb_ = V + (long long)b * T * ldv + (long long)h * HD;
  float qf[KP];
#pragma unroll
  for (int kk = 0; kk < KP; ++kk) qf[kk] = qi < T ? qb_[(long long)qi * ldq + 2 * kk + hf] : 0.f;
  f32x16 o[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[d][r] = 0.f;
  const float c2 = scale * kF32Log2e;
  float m = -INFINITY, lsum = 0.f;
  const int kv_end = causal ? min(T, q0 + BQ) : T;
  typename F32Rows<HD>::template Regs<BKV> gk, gv;
  constexpr bool PF = HD == 64;   // (at 32 the prefetch registers cost a wave per SIMD)
  if (PF) {
    F32Rows<HD>::fetch(gk, kb_, ldk, 0, T);
    F32Rows<HD>::fetch(gv, vb_, ldv, 0, T);
  }
  for (int kv0 = 0; kv0 < kv_end; kv0 += BKV) {
    __syncthreads();
    if (!PF) {
      F32Rows<HD>::fetch(gk, kb_, ldk, kv0, T);
      F32Rows<HD>::fetch(gv, vb_, ldv, kv0, T);
    }
    F32Rows<HD>::put(sk, gk);
    F32Rows<HD>::put(sv, gv);
    __syncthreads();
    if (PF && kv0 + BKV < kv_end) {   // the next tile's loads fly under this tile's MFMAs
      F32Rows<HD>::fetch(gk, kb_, ldk, kv0 + BKV, T);
      F32Rows<HD>::fetch(gv, vb_, ldv, kv0 + BKV, T);
    }
    if (causal && kv0 > q0 + 32 * wave + 31) continue;   // wave-uniform: every key after every query
    f32x16 s[2];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
      for (int r = 0; r < 16; ++r) s[kh][r] = 0.f;
#pragma unroll
      for (int kk = 0; kk < KP; ++kk) s[kh] = MFMA_F32(sk[(32 * kh + r32) * LD + 2 * kk + hf], qf[kk], s[kh]);
    }
    // mask: key kv0 + 32 kh + 8 (r >> 2) + 4 hf + (r & 3) valid iff <= the query (causal) and < T
    float mx = -INFINITY;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kv0 + 32 * kh + 8 * (r >> 2) + 4 * hf + (r & 3);
        const bool ok = key < T && (!causal || key <= qi);
        s[kh][r] = ok ? s[kh][r] * c2 : -INFINITY;
        mx = fmaxf(mx, s[kh][r]);
      }
    mx = pair_max_f(mx);
    const float mnew = fmaxf(m, mx);
    const float alpha = (m == -INFINITY) ? 0.f : exp2f(m - mnew);
    m = mnew;
    float ps = 0.f;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = (m == -INFINITY) ? 0.f : exp2f(s[kh][r] - m);
        s[kh][r] = p;
        ps += p;
      }
    lsum = lsum * alpha + pair_sum_f(ps);
#pragma unroll
    for (int d = 0; d < DT; ++d) o[d] *= alpha;
    // O^T[d][q] += V^T[d][key] P^T[key][q]
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int key = 32 * kh + 8 * (st >> 2) + 4 * hf + (st & 3);
#pragma unroll
        for (int d = 0; d < DT; ++d) o[d] = MFMA_F32(sv[key * LD + 32 * d + r32], s[kh][st], o[d]);
      }
  }
  if (qi < T) {
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    float* op = O + ((long long)b * T + qi) * ldo + (long long)h * HD;
#pragma unroll
    for (int d = 0; d < DT; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) op[32 * d + 8 * (r >> 2) + 4 * hf + (r & 3)] = o[d][r] * inv;
    if (hf == 0) LSE[(long long)bh * T + qi] = (m + log2f(lsum)) / kF32Log2e;
  }
}

// inverse RoPE of a gradient row fragment held as 16 registers per 32-wide d tile: register r
// of tile d is column 32 d + 8 (r >> 2) + 4 hf + (r & 3); d pairs with d + HD / 2 (tile + DT/2)
template <int HD>
__device__ __forceinline__ void inv_rope_tiles(f32x16 (&x)[HD / 32], const float* __restrict__ tr, int hf) {
  constexpr int DT = HD / 32;
  if constexpr (DT == 1) {
    // head_dim 32: column c < 16 (registers 0..7) pairs with c + 16 (register + 8), same tile
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int c = 8 * (r >> 2) + 4 * hf + (r & 3);
      const float cs = tr[c], sn = tr[HD / 2 + c];
      const float x1 = x[0][r], x2 = x[0][r + 8];
      x[0][r] = x1 * cs + x2 * sn;
      x[0][r + 8] = x2 * cs - x1 * sn;
    }
  } else {
#pragma unroll
    for (int d = 0; d < DT / 2; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = 32 * d + 8 * (r >> 2) + 4 * hf + (r & 3);
        const float cs = tr[c], sn = tr[HD / 2 + c];
        const float x1 = x[d][r], x2 = x[d + DT / 2][r];
        x[d][r] = x1 * cs + x2 * sn;
        x[d + DT / 2][r] = x2 * cs - x1 * sn;
      }
  }
}

// dQ (query on the lane) + the row constants of dK/dV: NDEL = -delta, LSN = -lse (fp32 path:
// p = exp(scale S - lse) computed directly).  BPQ: per-(b, h, query block, wave) column sums.
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_dq_f32_k(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
    const float* __restrict__ dO, const float* __restrict__ Og, const float* __restrict__ LSE,
    float* __restrict__ NDEL, float* __restrict__ dQ, int T, int H, long long ldq, long long ldk, long long ldv,
    long long lddo, long long ldo, long long lddq, float scale, int causal, const int64_t* __restrict__ rpos,
    const float* __restrict__ rtab, float* __restrict__ BPQ) {
  constexpr int BQ = 128, BKV = 64, KP = HD / 2, DT = HD / 32, LD = HD + 1;
  __shared__ float sk[BKV * LD], sv[BKV * LD];
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int qb = gridDim.x - 1 - blockIdx.x;
  const int q0 = qb * BQ, wave = threadIdx.x >> 6, l = lane_id(), r32 = l & 31, hf = l >> 5;
  const int qi = q0 + 32 * wave + r32;
  const long long rowq = (long long)b * T + qi;
  float qf[KP], df[KP];
  float dsum = 0.f;
#pragma unroll
  for (int kk = 0; kk < KP; ++kk) {
    const bool ok = qi < T;
    qf[kk] = ok ? Q[rowq * ldq + (long long)h * HD + 2 * kk + hf] : 0.f;
    df[kk] = ok ? dO[rowq * lddo + (long long)h * HD + 2 * kk + hf] : 0.f;
    dsum += ok ? df[kk] * Og[rowq * ldo + (long long)h * HD + 2 * kk + hf] : 0.f;
  }
  const float delta = pair_sum_f(dsum);
  const float lse = qi < T ? LSE[(long long)bh * T + qi] : 0.f;
  if (qi < T && hf == 0) NDEL[(long long)bh * T + qi] = -delta;
  const float* kb_ = K + (long long)b * T * ldk + (long long)h * HD;
  const float* vb_ = V + (long long)b * T * ldv + (long long)h * HD;
  f32x16 dq[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[d][r] = 0.f;
  const int kv_end = causal ? min(T, q0 + BQ) : T;
  const float lse2 = lse * kF32Log2e, c2 = scale * kF32Log2e;   // p = exp2(c2 S - lse log2 e)
  typename F32Rows<HD>::template Regs<BKV> gk, gv;
  constexpr bool PF = HD == 64;
  if (PF) {
    F32Rows<HD>::fetch(gk, kb_, ldk, 0, T);
    F32Rows<HD>::fetch(gv, vb_, ldv, 0, T);
  }
  for (int kv0 = 0; kv0 < kv_end; kv0 += BKV) {
    __syncthreads();
    if (!PF) {
      F32Rows<HD>::fetch(gk, kb_, ldk, kv0, T);
      F32Rows<HD>::fetch(gv, vb_, ldv, kv0, T);
    }
    F32Rows<HD>::put(sk, gk);
    F32Rows<HD>::put(sv, gv);
    __syncthreads();
    if (PF && kv0 + BKV < kv_end) {
      F32Rows<HD>::fetch(gk, kb_, ldk, kv0 + BKV, T);
      F32Rows<HD>::fetch(gv, vb_, ldv, kv0 + BKV, T);
    }
    if (causal && kv0 > q0 + 32 * wave + 31) continue;
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      f32x16 s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[r] = 0.f;
        dp[r] = 0.f;
      }
#pragma unroll
      for (int kk = 0; kk < KP; ++kk) {
        s = MFMA_F32(sk[(32 * kh + r32) * LD + 2 * kk + hf], qf[kk], s);
        dp = MFMA_F32(sv[(32 * kh + r32) * LD + 2 * kk + hf], df[kk], dp);
      }
      // dS^T = P^T (dP^T - delta), P^T = exp(scale S^T - lse), masked
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kv0 + 32 * kh + 8 * (r >> 2) + 4 * hf + (r & 3);
        const bool ok = key < T && qi < T && (!causal || key <= qi);
        const float p = ok ? exp2f(s[r] * c2 - lse2) : 0.f;
        s[r] = p * (dp[r] - delta);
      }
      // dQ^T[d][q] += K^T[d][key] dS^T[key][q]
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int key = 32 * kh + 8 * (st >> 2) + 4 * hf + (st & 3);
#pragma unroll
        for (int d = 0; d < DT; ++d) dq[d] = MFMA_F32(sk[key * LD + 32 * d + r32], s[st], dq[d]);
      }
    }
  }
#pragma unroll
  for (int d = 0; d < DT; ++d) dq[d] *= scale;
  if (rpos && qi < T) inv_rope_tiles<HD>(dq, rtab + rpos[(long long)b * T + qi] * HD, hf);
  if (qi < T) {
    float* p = dQ + rowq * lddq + (long long)h * HD;
#pragma unroll
    for (int d = 0; d < DT; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) p[32 * d + 8 * (r >> 2) + 4 * hf + (r & 3)] = dq[d][r];
  }
  if (BPQ) {   // column sums over the wave's 32 queries (transpose reduction, fixed order)
    const long long prow = (((long long)h * (gridDim.y / H) + b) * gridDim.x + qb) * 4 + wave;
    constexpr int NV = DT * 16, NP = NV < 32 ? 32 : NV;   // (head_dim 32: padded with zeros)
    float w[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) w[i] = (i < NV && qi < T) ? dq[i / 16 % DT][i % 16] : 0.f;
    lane32_sums(w, r32);
#pragma unroll
    for (int j = 0; j < NP / 32; ++j) {
      const int rr = r32 * (NP / 32) + j, r = rr & 15;
      if (rr < NV) BPQ[prow * HD + 32 * (rr >> 4) + 8 * (r >> 2) + 4 * hf + (r & 3)] = w[j];
    }
  }
}

// dK / dV (key on the lane): S = Q K^T with the queries as C rows; P = exp(scale S - lse[q]),
// dS = P (dP - delta[q]); dV^T += dO^T P, dK^T += Q^T dS with step s = 4 g + j reading the
// query 8 g + 4 hf + j of the stage.
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_dkdv_f32_k(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
    const float* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ NDEL,
    float* __restrict__ dK, float* __restrict__ dV, int T, int H, long long ldq, long long ldk, long long ldv,
    long long lddo, long long lddk, long long lddv, float scale, int causal, const int64_t* __restrict__ rpos,
    const float* __restrict__ rtab, float* __restrict__ BPK, float* __restrict__ BPV) {
  constexpr int BK = 128, BQ = 64, KP = HD / 2, DT = HD / 32, LD = HD + 1;
  __shared__ float sq[BQ * LD], sdo[BQ * LD], sl[BQ], sd[BQ];
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int kb = blockIdx.x;   // light (causal) blocks last
  const int k0 = kb * BK, wave = threadIdx.x >> 6, l = lane_id(), r32 = l & 31, hf = l >> 5;
  const int key = k0 + 32 * wave + r32;
  const long long rowk = (long long)b * T + key;
  float kf[KP], vf[KP];
#pragma unroll
  for (int kk = 0; kk < KP; ++kk) {
    kf[kk] = key < T ? K[rowk * ldk + (long long)h * HD + 2 * kk + hf] : 0.f;
    vf[kk] = key < T ? V[rowk * ldv + (long long)h * HD + 2 * kk + hf] : 0.f;
  }
  const float* qb_ = Q + (long long)b * T * ldq + (long long)h * HD;
  const float* dob_ = dO + (long long)b * T * lddo + (long long)h * HD;
  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dk[d][r] = 0.f;
      dv[d][r] = 0.f;
    }
  const int qstart = causal ? (k0 / BQ) * BQ : 0;
  const float c2 = scale * kF32Log2e;   // p = exp2(c2 S - lse log2 e)
  typename F32Rows<HD>::template Regs<BQ> gq, gd;
  float gl = 0.f, gdl = 0.f;
  auto fetch_tile = [&](int q0_) {
    F32Rows<HD>::fetch(gq, qb_, ldq, q0_, T);
    F32Rows<HD>::fetch(gd, dob_, lddo, q0_, T);
    if (threadIdx.x < BQ) {
      const int q = q0_ + threadIdx.x;
      gl = q < T ? LSE[(long long)bh * T + q] * kF32Log2e : 0.f;
      gdl = q < T ? -NDEL[(long long)bh * T + q] : 0.f;
    }
  };
  // (head_dim 64 only: at 32 the prefetch registers cost the second wave per SIMD, at 128
  // they spill)
  constexpr bool PF = HD == 64;
  if (PF && qstart < T) fetch_tile(qstart);
  for (int q0 = qstart; q0 < T; q0 += BQ) {
    __syncthreads();
    if (!PF) fetch_tile(q0);
    F32Rows<HD>::put(sq, gq);
    F32Rows<HD>::put(sdo, gd);
    if (threadIdx.x < BQ) {
      sl[threadIdx.x] = gl;
      sd[threadIdx.x] = gdl;
    }
    __syncthreads();
    if (PF && q0 + BQ < T) fetch_tile(q0 + BQ);   // the next tile's loads fly under this tile's MFMAs
    if (causal && q0 + BQ - 1 < k0 + 32 * wave) continue;   // every query before every key
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      f32x16 s, dp;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[r] = 0.f;
        dp[r] = 0.f;
      }
#pragma unroll
      for (int kk = 0; kk < KP; ++kk) {
        s = MFMA_F32(sq[(32 * qh + r32) * LD + 2 * kk + hf], kf[kk], s);
        dp = MFMA_F32(sdo[(32 * qh + r32) * LD + 2 * kk + hf], vf[kk], dp);
      }
      f32x16 pd;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ql = 32 * qh + 8 * (r >> 2) + 4 * hf + (r & 3), q = q0 + ql;
        const bool ok = key < T && q < T && (!causal || key <= q);
        const float p = ok ? exp2f(s[r] * c2 - sl[ql]) : 0.f;
        s[r] = p;
        pd[r] = p * (dp[r] - sd[ql]);
      }
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int ql = 32 * qh + 8 * (st >> 2) + 4 * hf + (st & 3);
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          dv[d] = MFMA_F32(sdo[ql * LD + 32 * d + r32], s[st], dv[d]);
          dk[d] = MFMA_F32(sq[ql * LD + 32 * d + r32], pd[st], dk[d]);
        }
      }
    }
  }
#pragma unroll
  for (int d = 0; d < DT; ++d) dk[d] *= scale;
  if (rpos && key < T) inv_rope_tiles<HD>(dk, rtab + rpos[rowk] * HD, hf);
  if (key < T) {
    float* pk = dK + rowk * lddk + (long long)h * HD;
    float* pv = dV + rowk * lddv + (long long)h * HD;
#pragma unroll
    for (int d = 0; d < DT; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int c = 32 * d + 8 * (r >> 2) + 4 * hf + (r & 3);
        pk[c] = dk[d][r];
        pv[c] = dv[d][r];
      }
  }
  if (BPK) {   // column sums over the wave's 32 keys (transpose reduction, fixed order)
    const long long row = (((long long)h * (gridDim.y / H) + b) * gridDim.x + kb) * 4 + wave;
    constexpr int NV = DT * 16, NP = NV < 32 ? 32 : NV;   // (head_dim 32: padded with zeros)
    float wk[NP], wv[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      wk[i] = (i < NV && key < T) ? dk[i / 16 % DT][i % 16] : 0.f;
      wv[i] = (i < NV && key < T) ? dv[i / 16 % DT][i % 16] : 0.f;
    }
    lane32_sums(wk, r32);
    lane32_sums(wv, r32);
#pragma unroll
    for (int j = 0; j < NP / 32; ++j) {
      const int rr = r32 * (NP / 32) + j, r = rr & 15;
      if (rr < NV) {
        const int cc = 32 * (rr >> 4) + 8 * (r >> 2) + 4 * hf + (r & 3);
        BPK[row * HD + cc] = wk[j];
        BPV[row * HD + cc] = wv[j];
      }
    }
  }
}

// C (+)= sum over the S slabs (split order: deterministic); vectorised by 4 where aligned
template <typename TO>
__global__ __launch_bounds__(256) void splitk_sum_f32_k(const float* __restrict__ ws, TO* __restrict__ C,
                                                        const float* __restrict__ bias, int M, int N, long long ldc,
                                                        int S, int accumulate) {
  const long long n = (long long)M * N;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    float acc = 0.f;
    for (int sp = 0; sp < S; ++sp) acc += ws[sp * n + i];
    const long long r = i / N, c = i % N;
    if (bias) acc += bias[c];
    TO* p = C + r * ldc + c;
    *p = from_f<TO>(accumulate ? to_f(*p) + acc : acc);
  }
}

// column sums of the per-wave partial rows: out[seg][h][c] = sum over R rows (fixed order)
__global__ __launch_bounds__(256) void colsum_parts_f32_k(const float* __restrict__ P, float* __restrict__ out,
                                                          int R, int HD, int H) {
  // blockIdx.x = h * HD + c
  const int h = blockIdx.x / HD, c = blockIdx.x % HD;
  __shared__ float red[256];
  float s = 0.f;
  for (int r = threadIdx.x; r < R; r += 256) s += P[((long long)h * R + r) * HD + c];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[(long long)h * HD + c] = red[0];
}

}  // namespace dpfs

using namespace dpfs;

// K-splits of an M x N x K fp32 GEMM: enough workgroups to fill the chip (~4 per CU) when the
// output tiles alone do not, each split at least 512 deep.
extern "C" int dpfs_gemm_f32_splits(int M, int N, int K) {
  const long long tiles = (long long)((M + kF32BM - 1) / kF32BM) * ((N + kF32BM - 1) / kF32BM);
  long long sp = (1024 + tiles - 1) / tiles;
  sp = std::min<long long>(sp, std::max(1, K / 512));
  return (int)std::max<long long>(1, std::min<long long>(sp, 64));
}

// layout: 0 = NT (a[M][K], b[N][K]), 1 = NN (a[M][K], b[K][N]), 2 = TN (a[K][M], b[K][N]).
// ws: splits * M * N floats when dpfs_gemm_f32_splits > 1 (else unused, may be null).
template <typename TI, typename TO>
static void gemm_generic(int layout, const TI* A, const TI* B, TO* C, const float* bias, int M, int N, int K,
                         long long lda, long long ldb, long long ldc, int accumulate, float* ws, hipStream_t s) {
  if (M <= 0 || N <= 0) return;
  const int tiles = ((M + kF32BM - 1) / kF32BM) * ((N + kF32BM - 1) / kF32BM);
  constexpr int VA = sizeof(TI) == 4 ? 16 : 8;   // bytes of a 4-element vector load
  const bool va = ((uintptr_t)A % VA == 0) && lda % 4 == 0, vb = ((uintptr_t)B % VA == 0) && ldb % 4 == 0;
  const int S = ws ? dpfs_gemm_f32_splits(M, N, K) : 1;
  const int kps = S > 1 ? ((K + S - 1) / S + kF32BK - 1) / kF32BK * kF32BK : K;
  const int Sx = S > 1 ? (K + kps - 1) / kps : 1;
  dim3 grid(tiles, Sx);
  const long long slab = (long long)M * N;
#define GF32(AK_, BK_)                                                                                              \
  do {                                                                                                              \
    if (Sx > 1)                                                                                                     \
      gemm_f32_k<AK_, BK_, TI, float><<<grid, 256, 0, s>>>(A, B, ws, nullptr, M, N, K, lda, ldb, N, 0, va, vb, kps,  \
                                                            slab);                                                  \
    else                                                                                                            \
      gemm_f32_k<AK_, BK_, TI, TO><<<grid, 256, 0, s>>>(A, B, C, bias, M, N, K, lda, ldb, ldc, accumulate, va, vb,   \
                                                         kps, slab);                                                \
  } while (0)
  if (layout == 0) GF32(true, true);
  else if (layout == 1) GF32(true, false);
  else GF32(false, false);
#undef GF32
  if (Sx > 1) {
    const int blocks = (int)std::min<long long>((slab + 255) / 256, 4096);
    splitk_sum_f32_k<TO><<<blocks, 256, 0, s>>>(ws, C, bias, M, N, ldc, Sx, accumulate);
  }
}

// in_bf16 / out_bf16: operand / output storage (fp32 otherwise)
extern "C" void dpfs_gemm_f32(int layout, const void* A, const void* B, void* C, const float* bias, int M, int N,
                              int K, long long lda, long long ldb, long long ldc, int accumulate, float* ws,
                              int in_bf16, int out_bf16, hipStream_t s) {
  if (in_bf16 && out_bf16)
    gemm_generic<bf16, bf16>(layout, (const bf16*)A, (const bf16*)B, (bf16*)C, bias, M, N, K, lda, ldb, ldc,
                             accumulate, ws, s);
  else if (in_bf16)
    gemm_generic<bf16, float>(layout, (const bf16*)A, (const bf16*)B, (float*)C, bias, M, N, K, lda, ldb, ldc,
                              accumulate, ws, s);
  else
    gemm_generic<float, float>(layout, (const float*)A, (const float*)B, (float*)C, bias, M, N, K, lda, ldb, ldc,
                               accumulate, ws, s);
}

extern "C" int dpfs_attn_f32_supported_hd(int hd) { return hd == 32 || hd == 64 || hd == 128; }

#define F32_HD(HDV, ...)                                                         \
  do {                                                                           \
    if ((HDV) == 64) { constexpr int HD_ = 64; __VA_ARGS__; }                    \
    else if ((HDV) == 128) { constexpr int HD_ = 128; __VA_ARGS__; }             \
    else if ((HDV) == 32) { constexpr int HD_ = 32; __VA_ARGS__; }               \
  } while (0)

extern "C" void dpfs_attn_fwd_f32(const float* q, const float* k, const float* v, float* o, float* lse, int B, int T,
                                  int H, int hd, long long ldq, long long ldk, long long ldv, long long ldo,
                                  float scale, int causal, hipStream_t s) {
  dim3 grid((T + 127) / 128, B * H);
  F32_HD(hd, attn_fwd_f32_k<HD_><<<grid, 256, 0, s>>>(q, k, v, o, lse, T, H, ldq, ldk, ldv, ldo, scale, causal));
}

// ws: B * H * T floats (-delta) + (bias) partial rows.  Returns 1 when dbias was written.
extern "C" long long dpfs_attn_bwd_f32_ws(int B, int T, int H, int hd, int bias) {
  const long long nqb = (T + 127) / 128, nkb = (T + 127) / 128;
  return (long long)B * H * T + (bias ? (long long)H * B * (nqb + 2 * nkb) * 4 * hd : 0);
}
extern "C" int dpfs_attn_bwd_f32(const float* dout, const float* q, const float* k, const float* v, const float* o,
                                 const float* lse, float* ws, float* dq, float* dk, float* dv, int B, int T, int H,
                                 int hd, long long lddo, long long ldq, long long ldk, long long ldv, long long ldo,
                                 long long lddq, long long lddk, long long lddv, float scale, int causal,
                                 const int64_t* rpos, const float* rtab, float* dbias, hipStream_t s) {
  const long long nqb = (T + 127) / 128, nkb = (T + 127) / 128;
  float* ndel = ws;
  float* pq = dbias ? ws + (long long)B * H * T : nullptr;
  float* pk = dbias ? pq + (long long)H * B * nqb * 4 * hd : nullptr;
  float* pv = dbias ? pk + (long long)H * B * nkb * 4 * hd : nullptr;
  dim3 gq((unsigned)nqb, B * H), gk((unsigned)nkb, B * H);
  F32_HD(hd, attn_bwd_dq_f32_k<HD_><<<gq, 256, 0, s>>>(q, k, v, dout, o, lse, ndel, dq, T, H, ldq, ldk, ldv, lddo,
                                                            ldo, lddq, scale, causal, rpos, rtab, pq));
  F32_HD(hd, attn_bwd_dkdv_f32_k<HD_><<<gk, 256, 0, s>>>(q, k, v, dout, lse, ndel, dk, dv, T, H, ldq, ldk, ldv, lddo,
                                                              lddk, lddv, scale, causal, rpos, rtab, pk, pv));
  if (dbias) {
    colsum_parts_f32_k<<<H * hd, 256, 0, s>>>(pq, dbias, (int)(B * nqb * 4), hd, H);
    colsum_parts_f32_k<<<H * hd, 256, 0, s>>>(pk, dbias + (long long)H * hd, (int)(B * nkb * 4), hd, H);
    colsum_parts_f32_k<<<H * hd, 256, 0, s>>>(pv, dbias + 2LL * H * hd, (int)(B * nkb * 4), hd, H);
    return 1;
  }
  return 0;
}
