// bf16 MFMA GEMM for gfx950 (MI355X) — the three layouts of a tensor-parallel linear.
//
//   C[m][n] = sum_k A(m,k) B(k,n)       fp32 accumulate in MFMA accumulators
//
//   layout  A(m,k)            B(k,n)            use
//   NT      a[m*lda + k]      b[n*ldb + k]      forward   y  = x W^T (+bias)       (F.linear)
//   NN      a[m*lda + k]      b[k*ldb + n]      dgrad     dx = dy W
//   TN      a[k*lda + m]      b[k*ldb + n]      wgrad     dW = dy^T x   (fp32 out, split-K)
//
// Reference call sites: models/layers.py:49,93 (F.linear) and their autograd backward
// (SURVEY.md K8/K9).  Two kernels live here: gemm2_k (v2, the default: 256x256 / 256x128
// tiles, 8 waves, LDS-DMA staging, split-K; described at its definition) and gemm_k (v1,
// kept for small-output wgrads where its 128x128 tile fills the chip better).  The
// selection heuristics below were derived from tools/tune_gemm.py sweeps on MI355X.
// v1 design (CDNA HIP guide §5):
//  * 128x128x64 block tile, 256 threads = 4 waves in 2x2, each wave 64x64 = 4x4 tiles of
//    v_mfma_f32_16x16x32_bf16 (16 accumulators x 4 regs);
//  * operands staged global -> registers (16-byte loads) -> LDS, double-buffered LDS with the
//    next tile's global loads issued BEFORE the current tile's MFMAs and written AFTER them
//    (async-STAGE split, T14), one barrier per K-step;
//  * K-contiguous operand tiles [rows][64] with an XOR chunk swizzle (chunk ^ row&7) read by
//    ds_read_b128; MN-contiguous tiles [64][128] (the transposed operands of dgrad/wgrad)
//    swizzled (chunk ^ 2h(row)) and read with the CDNA4 hardware-transpose read
//    ds_read_b64_tr_b16 (T10) — no transpose kernels, no scalar LDS traffic;
//  * bijective XCD-aware block remap (T1) with n fastest, so the blocks of one XCD share the
//    weight panel in their L2;
//  * edges: rows/cols masked on load (zero fill) and store; the contiguous dim of each
//    operand must be a multiple of 8 (16-byte vectors);
//  * split-K over blockIdx.y for the skinny-output wgrad: fp32 slabs + fixed-order reduction
//    (deterministic, no float atomics).
#include "common.h"

#include <algorithm>

namespace dpfs {

constexpr int BM = 128, BN = 128, BKK = 64;
constexpr int kTileBytes = 128 * 64 * 2;  // 16 KiB per operand tile

// MN-major swizzle: rows read together by one ds_read_b64_tr_b16 half-wave are
// {b..b+3, b+8..b+11}; h() maps them to 8 distinct chunk pairs -> conflict-free.
__device__ __forceinline__ int mn_h(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

__device__ __forceinline__ int kmaj_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }
__device__ __forceinline__ int mnmaj_off(int row, int chunk) { return row * 256 + ((chunk ^ (mn_h(row) << 1)) << 4); }

template <bool KMAJ>
__device__ __forceinline__ void g2r(const bf16* __restrict__ P, int ld, int R, int K, int r0, int k0, u32x4 (&reg)[4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = tid + 256 * i;
    int row, c;
    const bf16* src;
    bool ok;
    if (KMAJ) {
      row = q >> 3; c = q & 7;
      ok = (r0 + row < R) && (k0 + c * 8 < K);
      src = P + (long long)(r0 + row) * ld + k0 + c * 8;
    } else {
      row = q >> 4; c = q & 15;
      ok = (k0 + row < K) && (r0 + c * 8 < R);
      src = P + (long long)(k0 + row) * ld + r0 + c * 8;
    }
    u32x4 v = {0u, 0u, 0u, 0u};
    if (ok) v = *reinterpret_cast<const u32x4*>(src);
    reg[i] = v;
  }
}

template <bool KMAJ>
__device__ __forceinline__ void r2lds(char* lds, const u32x4 (&reg)[4]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = tid + 256 * i;
    const int off = KMAJ ? kmaj_off(q >> 3, q & 7) : mnmaj_off(q >> 4, q & 15);
    *reinterpret_cast<u32x4*>(lds + off) = reg[i];
  }
}

// Fragment of the 16x16x32 MFMA operand: lane l holds X[rb + (l&15)][kb + 8(l>>4) + j], j<8,
// where X is A (row = m) or B^T (row = n).
template <bool KMAJ>
__device__ __forceinline__ bf16x8 frag(const char* lds, int rb, int kb) {
  const int l = lane_id();
  if (KMAJ) {
    const int row = rb + (l & 15);
    const int chunk = (kb >> 3) + (l >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + kmaj_off(row, chunk));
  } else {
    const int i = l & 15, q = i >> 2, p = i & 3;
    const int col = rb + 4 * p;
    const int chunk = col >> 3;
    s16x4 lo, hi;
    {
      const int k = kb + 8 * (l >> 4) + q;
      lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(lds + mnmaj_off(k, chunk) + (p & 1) * 8));
    }
    {
      const int k = kb + 8 * (l >> 4) + 4 + q;
      hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(lds + mnmaj_off(k, chunk) + (p & 1) * 8));
    }
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// OUT: 0 = bf16 C (+ optional fp32 bias[n]); 1 = fp32 C slab (split-K partial or final).
template <bool AK, bool BKM, int OUT>
__global__ __launch_bounds__(256, 2) void gemm_k(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                 void* __restrict__ C, const float* __restrict__ bias, int M, int N,
                                                 int K, int lda, int ldb, int ldc, int k_per_split,
                                                 long long slab_stride) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * kTileBytes];
  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int tm = wg / tiles_n, tn = wg % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = blockIdx.y * k_per_split;
  const int kend = min(K, kbeg + k_per_split);

  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int l = lane_id();

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  u32x4 ra[4], rb[4];
  const int nk = (kend - kbeg + BKK - 1) / BKK;
  if (nk > 0) {
    g2r<AK>(A, lda, M, kend, m0, kbeg, ra);
    g2r<BKM>(B, ldb, N, kend, n0, kbeg, rb);
    r2lds<AK>(smem, ra);
    r2lds<BKM>(smem + kTileBytes, rb);
  }
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    const char* la = smem + cur * 2 * kTileBytes;
    const char* lb = la + kTileBytes;
    const bool more = (t + 1) < nk;
    if (more) {
      const int k0 = kbeg + (t + 1) * BKK;
      g2r<AK>(A, lda, M, kend, m0, k0, ra);
      g2r<BKM>(B, ldb, N, kend, n0, k0, rb);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag<AK>(la, wm * 64 + i * 16, s * 32);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag<BKM>(lb, wn * 64 + j * 16, s * 32);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      char* na = smem + (cur ^ 1) * 2 * kTileBytes;
      r2lds<AK>(na, ra);
      r2lds<BKM>(na + kTileBytes, rb);
    }
    __syncthreads();
  }

  // Epilogue: C/D map of 16x16 MFMA: col = lane&15, row = 4*(lane>>4) + j.
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wn * 64 + j * 16 + (l & 15);
      if (col >= N) continue;
      float bv = 0.f;
      if (OUT == 0 && bias) bv = bias[col];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 64 + i * 16 + 4 * (l >> 4) + r;
        if (row < M) {
          if (OUT == 0) {
            reinterpret_cast<bf16*>(C)[(long long)row * ldc + col] = (bf16)(acc[i][j][r] + bv);
          } else {
            reinterpret_cast<float*>(C)[blockIdx.y * slab_stride + (long long)row * ldc + col] = acc[i][j][r];
          }
        }
      }
    }
  }
}

// out[i] (+)= sum_s slab[s][i]  (fixed order), float4 vectorised; n % 4 == 0.
__global__ __launch_bounds__(256) void splitk_reduce_k(const float* __restrict__ slabs, float* __restrict__ out,
                                                       long long n, int S, int accumulate) {
  for (long long i = (blockIdx.x * (long long)blockDim.x + threadIdx.x) * 4; i < n;
       i += (long long)gridDim.x * blockDim.x * 4) {
    f32x4 s = accumulate ? *reinterpret_cast<const f32x4*>(out + i) : (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < S; ++k) s += *reinterpret_cast<const f32x4*>(slabs + k * n + i);
    *reinterpret_cast<f32x4*>(out + i) = s;
  }
}


// ======================================================================== GEMM v2 ====
// 256x256 (or 256x128) x 64 block tile, 512 threads = 8 waves, LDS-DMA staging.
//  * operands go HBM -> LDS with buffer_load_dwordx4 ... lds (no VGPR round trip, no
//    ds_write: the register-staged v1 was bound by ds_write_b128 throughput); the LDS image
//    is lane-linear per 1 KiB DMA piece, so the XOR swizzles are applied on the SOURCE
//    address (rule 21: linear dest + swizzled source + the same swizzle on read);
//  * tails: a per-lane offset past the buffer descriptor's num_records returns zeros, so K
//    tails contribute nothing and out-of-range rows never fault (no branches in the loop);
//  * 2 LDS stages: the DMA of tile t+1 is in flight while tile t is multiplied; counted
//    `s_waitcnt vmcnt(pieces of t+1)` + raw s_barrier (never vmcnt(0) in steady state);
//  * MFMA operands swapped (acc = W-frag x X-frag) so each lane owns 4 consecutive output
//    columns of one row: bf16x4 / f32x4 vector stores and a vector bias load.
// Issue the DMA of one operand tile (R rows/cols x 64 k) into LDS at `tile`.
template <bool KMAJ, int R, int NWV = 8>
__device__ __forceinline__ void issue_tile(__amdgpu_buffer_rsrc_t rs, char* tile, int r0, int k0, int ld, int K) {
  const int l = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int i = 0; i < R / 8 / NWV; ++i) {
    const int j = wave + NWV * i;  // 1 KiB piece index
    unsigned off;
    if (KMAJ) {
      const int row = 8 * j + (l >> 3);
      const int c = (l & 7) ^ ((l >> 3) & 7);
      const int k = k0 + c * 8;
      off = (k < K) ? (unsigned)(((long long)(r0 + row) * ld + k) * 2) : kOOB;
    } else {
      constexpr int CPR = R / 8;
      const int lin = j * 64 + l;
      const int row = lin / CPR;
      const int c = (lin % CPR) ^ (mn_h(row) << 1);
      const int k = k0 + row;
      off = (k < K) ? (unsigned)(((long long)k * ld + r0 + c * 8) * 2) : kOOB;
    }
    dma16(rs, tile + j * 1024, off);
  }
}

// One 1 KiB DMA piece (index i < R/64) of issue_tile, for schedules that spread the
// pieces between MFMAs.
template <bool KMAJ, int R, int NWV = 8>
__device__ __forceinline__ void issue_piece(__amdgpu_buffer_rsrc_t rs, char* tile, int r0, int k0, int ld, int K,
                                            int i) {
  const int l = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = wave + NWV * i;
  unsigned off;
  if (KMAJ) {
    const int row = 8 * j + (l >> 3);
    const int c = (l & 7) ^ ((l >> 3) & 7);
    const int k = k0 + c * 8;
    off = (k < K) ? (unsigned)(((long long)(r0 + row) * ld + k) * 2) : kOOB;
  } else {
    constexpr int CPR = R / 8;
    const int lin = j * 64 + l;
    const int row = lin / CPR;
    const int c = (lin % CPR) ^ (mn_h(row) << 1);
    const int k = k0 + row;
    off = (k < K) ? (unsigned)(((long long)k * ld + r0 + c * 8) * 2) : kOOB;
  }
  dma16(rs, tile + j * 1024, off);
}

template <bool KMAJ, int R>
__device__ __forceinline__ bf16x8 frag2(const char* lds, int rb, int kb) {
  const int l = lane_id();
  if (KMAJ) {
    const int row = rb + (l & 15);
    const int chunk = (kb >> 3) + (l >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((chunk ^ (row & 7)) << 4));
  } else {
    constexpr int RB = R * 2;
    const int i = l & 15, q = i >> 2, p = i & 3;
    const int chunk = (rb + 4 * p) >> 3;
    const int k_lo = kb + 8 * (l >> 4) + q;
    const int k_hi = k_lo + 4;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(lds + k_lo * RB + ((chunk ^ (mn_h(k_lo) << 1)) << 4) + (p & 1) * 8));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(lds + k_hi * RB + ((chunk ^ (mn_h(k_hi) << 1)) << 4) + (p & 1) * 8));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// Optional RoPE (rotate-half, head_dim 64) applied in the NT epilogue to output columns
// < cols (the q and k heads of a packed QKV projection); pos[m] indexes tab[maxlen][64]
// = [cos | sin].  Each wave's 64 output columns are exactly one head, and with the swapped
// MFMA layout the rotation partner of column d (d + 32) sits in the same lane (tile j+2), so
// the rotation is pure register math — no separate RoPE pass over the QKV activations.
struct RopeArgs {
  const int64_t* pos;
  const float* tab;
  int cols;
  int hd = 64;
};

template <int PIECES, int NSTAGE>
__device__ __forceinline__ void wait_tile(int remaining_after) {
  // Tiles issued after the one we need: min(NSTAGE-2, remaining_after); each = PIECES DMAs.
  if (NSTAGE >= 3 && remaining_after >= 1) {
    if (NSTAGE >= 4 && remaining_after >= 2) wait_vmcnt<2 * PIECES>();
    else wait_vmcnt<PIECES>();
  } else {
    wait_vmcnt<0>();
  }
}

// OUT: 0 = bf16 C (+bias); 1 = fp32 C / split-K slab.
// SCHED: 0 = all DMA pieces right after the barrier; 1 = after the first k-half's MFMAs;
// 2 = one piece after each MFMA row of the first k-half (spreads the DMA issue cost).
// NWV: waves per workgroup.  8 (two waves per SIMD) is what runs: a 4-wave variant with
// 128x128 wave tiles (accumulators in AGPRs, one wave per SIMD) measured 20-30 % slower
// without hand-placed software pipelining (profiles/r1_gemm_sched_sweep.log).
template <int BM_, int BN_, int WAVES_M, int NSTAGE, bool AK, bool BKM, int OUT, int SCHED = 0, int NWV = 8>
__global__ __launch_bounds__(64 * NWV, NWV == 8 ? 2 : 1) void gemm2_k(const bf16* __restrict__ A,
                                                                  const bf16* __restrict__ B, void* __restrict__ C,
                                                                  const float* __restrict__ bias, int M, int N, int K,
                                                                  int lda, int ldb, int ldc, int k_per_split,
                                                                  long long slab_stride, unsigned a_bytes,
                                                                  unsigned b_bytes, RopeArgs rope) {
  constexpr int WAVES_N = NWV / WAVES_M;
  constexpr int WM = BM_ / WAVES_M, WN = BN_ / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_BYTES = BM_ * 128, B_BYTES = BN_ * 128, STAGE = A_BYTES + B_BYTES;
  constexpr int PA = BM_ / 8 / NWV, PB = BN_ / 8 / NWV;  // DMA pieces per wave per K-step
  constexpr int PIECES = PA + PB;
  __shared__ __attribute__((aligned(1024))) char smem[NSTAGE * STAGE];

  const int tiles_n = (N + BN_ - 1) / BN_;
  const int tiles_m = (M + BM_ - 1) / BM_;
  const int nwg = tiles_m * tiles_n;
  // XCD-aware over the whole (tile, split) grid: the hardware deals linear block ids to the 8
  // XCDs round-robin, so remap the LINEAR id (a split-K grid's tile count is rarely a multiple
  // of 8); every XCD then holds a contiguous run of (split, tile) pairs: the tiles of one
  // K-split, which stream the same K-slab of both operands, share that XCD's L2.
  const int lin = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, nwg * gridDim.y);
  const int split = lin / nwg;
  const int wg = lin - split * nwg;
  const int tm = wg / tiles_n, tn = wg % tiles_n;
  const int m0 = tm * BM_, n0 = tn * BN_;
  const int kbeg = split * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  const int nk = kend > kbeg ? (kend - kbeg + 63) / 64 : 0;

  const int wave = threadIdx.x >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int l = lane_id();

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, (int)b_bytes, 0x00020000);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // Prologue: NSTAGE-1 tiles in flight.
#pragma unroll
  for (int s0 = 0; s0 < NSTAGE - 1; ++s0) {
    if (s0 < nk) {
      char* st = smem + s0 * STAGE;
      issue_tile<AK, BM_, NWV>(ra, st, m0, kbeg + s0 * 64, lda, kend);
      issue_tile<BKM, BN_, NWV>(rb, st + A_BYTES, n0, kbeg + s0 * 64, ldb, kend);
    }
  }
  int cur = 0;
  for (int t = 0; t < nk; ++t) {
    wait_tile<PIECES, NSTAGE>(nk - 1 - t);
    __builtin_amdgcn_s_barrier();  // tile t landed for all waves; tile t-1's buffer is free
    const bool more = t + NSTAGE - 1 < nk;
    int nb = cur + NSTAGE - 1;
    if (nb >= NSTAGE) nb -= NSTAGE;
    char* nst = smem + nb * STAGE;
    const int k1 = kbeg + (t + NSTAGE - 1) * 64;
    if (SCHED == 0 && more) {
      issue_tile<AK, BM_, NWV>(ra, nst, m0, k1, lda, kend);
      issue_tile<BKM, BN_, NWV>(rb, nst + A_BYTES, n0, k1, ldb, kend);
    }
    const char* la = smem + cur * STAGE;
    const char* lb = la + A_BYTES;
    auto piece = [&](int q) {
      if (q < PA) issue_piece<AK, BM_, NWV>(ra, nst, m0, k1, lda, kend, q);
      else issue_piece<BKM, BN_, NWV>(rb, nst + A_BYTES, n0, k1, ldb, kend, q - PA);
    };
    if constexpr (SCHED == 4) {
      // both k-halves' fragments read up front (the second half's reads land under the
      // first half's MFMAs); DMA pieces spread over the first half's MFMA rows.
      bf16x8 fa[2][TM], fb[2][TN];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[s][j] = frag2<BKM, BN_>(lb, wn * WN + 16 * j, 32 * s);
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[s][i] = frag2<AK, BM_>(la, wm * WM + 16 * i, 32 * s);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[s][j], fa[s][i], acc[i][j], 0, 0, 0);
          if (s == 0 && more) {
#pragma unroll
            for (int q = 0; q < PIECES; ++q)
              if ((q * TM) / PIECES == i) piece(q);
          }
        }
        __builtin_amdgcn_s_setprio(0);
      }
    } else {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = frag2<AK, BM_>(la, wm * WM + 16 * i, 32 * s);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = frag2<BKM, BN_>(lb, wn * WN + 16 * j, 32 * s);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
        if (SCHED == 2 && s == 0 && more) {
          // spread PIECES DMA instructions over the TM MFMA rows of this k-half
#pragma unroll
          for (int q = 0; q < PIECES; ++q)
            if ((q * TM) / PIECES == i) piece(q);
        }
        if (SCHED == 3 && more) {
          // spread them over the MFMA rows of both k-halves
#pragma unroll
          for (int q = 0; q < PIECES; ++q)
            if ((q * 2 * TM) / PIECES == s * TM + i) piece(q);
        }
      }
      __builtin_amdgcn_s_setprio(0);
      if (SCHED == 1 && s == 0 && more) {
        issue_tile<AK, BM_, NWV>(ra, nst, m0, k1, lda, kend);
        issue_tile<BKM, BN_, NWV>(rb, nst + A_BYTES, n0, k1, ldb, kend);
      }
    }
    }
    cur = (cur + 1 == NSTAGE) ? 0 : cur + 1;
  }

  // Epilogue: acc[i][j] = C^T tile: lane holds C[m = .. + (l&15)][n = .. + 4g + r], r < 4.
  const int g = l >> 4;
  const int wcol0 = n0 + wn * WN;
  // RoPE needs each 64-column head inside one wave (WN % 64 == 0): head hg of the wave is
  // tiles 4hg..4hg+3 and column d's partner d + 32 is tile + 2 in the same lane.
  const bool do_rope = (OUT == 0) && (WN % 64 == 0) && rope.cols > 0 && wcol0 < rope.cols;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * WM + 16 * i + (l & 15);
    if (m >= M) continue;
    f32x4 v[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      v[j] = acc[i][j];
      const int n = wcol0 + 16 * j + 4 * g;
      if (OUT == 0 && bias && n < N) v[j] += *reinterpret_cast<const f32x4*>(bias + n);
    }
    if constexpr (OUT == 0 && WN % 64 == 0) {
      if (do_rope) {
        const float* tr = rope.tab + rope.pos[m] * 64;
#pragma unroll
        for (int hg = 0; hg < WN / 64; ++hg) {
          if (wcol0 + 64 * hg >= rope.cols) break;
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const f32x4 cs = *reinterpret_cast<const f32x4*>(tr + 16 * j + 4 * g);
            const f32x4 sn = *reinterpret_cast<const f32x4*>(tr + 32 + 16 * j + 4 * g);
            const f32x4 x1 = v[4 * hg + j], x2 = v[4 * hg + j + 2];
            v[4 * hg + j] = x1 * cs - x2 * sn;
            v[4 * hg + j + 2] = x2 * cs + x1 * sn;
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = wcol0 + 16 * j + 4 * g;
      if (n >= N) continue;
      if (OUT == 0) {
        bf16x4 o = {(bf16)v[j][0], (bf16)v[j][1], (bf16)v[j][2], (bf16)v[j][3]};
        *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(C) + (long long)m * ldc + n) = o;
      } else {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(C) + split * slab_stride + (long long)m * ldc + n) = v[j];
      }
    }
  }
}

// Second operand pair of a TN GEMM whose reduction dim is split over two buffers (the two
// ping-pong chunks' activations of a chunked training step): k < k_switch reads (A, B),
// k >= k_switch reads (A2, B2) at k - k_switch.  K-splits never straddle k_switch (the
// launcher checks it), so each work item reads one pair.  k_switch = INT_MAX: one pair.
struct Dual {
  const bf16* A2;
  const bf16* B2;
  int k_switch, lda2, ldb2;
  unsigned a2_bytes, b2_bytes;
};
constexpr Dual kNoDual = {nullptr, nullptr, 0x7fffffff, 0, 0, 0u, 0u};

// ============================================================= GEMM v3 (persistent) ====
// gemm2_k's 256-wide tile, made persistent: one workgroup per CU walks the (split, tile)
// items i = r, r + G, r + 2G, ... (r = XCD-remapped block id, G = grid), so the per-tile
// fixed cost the one-tile-per-workgroup kernel pays on short-K shapes (K = 768: ~40 % of its
// time on MI355X) overlaps the neighbouring tiles' MFMA work:
//  * the LAST K-step of an item issues the LDS-DMA of the NEXT item's first K-tile (the
//    stage the K-loop would have filled next), so the next item's operands are in flight
//    while this item's MFMAs drain and its epilogue stores issue — no pipeline restart;
//  * epilogue stores are buffer stores with out-of-range lanes dropped by the descriptor
//    bound (no per-lane branches): every wave issues exactly TM*TN stores, so the next
//    item's first wait is a counted `vmcnt(TM*TN)` that retires the prefetched tile without
//    waiting for the stores to drain;
//  * item order: grouped (GROUP_M tile rows, then the next tile column), and the XCD remap
//    makes the items running concurrently on one XCD a contiguous run = a GROUP_M x (32 /
//    GROUP_M) block of tiles sharing A rows and B columns in that XCD's L2.
// NSTAGE = 2 (two 64-deep K stages, 128 KiB LDS at 256x256), SCHED as gemm2_k (2 or 4).
template <int BM_, int BN_, int WAVES_M, bool AK, bool BKM, int OUT, int SCHED>
__global__ __launch_bounds__(512, 1) void gemmp_k(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                  void* __restrict__ C, const float* __restrict__ bias, int M, int N,
                                                  int K, int lda, int ldb, int ldc, int k_per_split, int splits,
                                                  long long slab_stride, unsigned a_bytes, unsigned b_bytes,
                                                  unsigned c_bytes, RopeArgs rope, int group_m, Dual dual) {
  constexpr int NWV = 8;
  constexpr int WAVES_N = NWV / WAVES_M;
  constexpr int WM = BM_ / WAVES_M, WN = BN_ / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_BYTES = BM_ * 128, B_BYTES = BN_ * 128, STAGE = A_BYTES + B_BYTES;
  constexpr int PA = BM_ / 8 / NWV, PB = BN_ / 8 / NWV;
  constexpr int PIECES = PA + PB;
  constexpr int STORES = TM * TN;
  static_assert(STORES < 64 && PIECES < 64, "vmcnt range");
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tiles_n = (N + BN_ - 1) / BN_;
  const int tiles_m = (M + BM_ - 1) / BM_;
  const int nwg = tiles_m * tiles_n;
  const int total = nwg * splits;
  const int G = gridDim.x;
  const int wave = threadIdx.x >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int l = lane_id();
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, (int)b_bytes, 0x00020000);
  const bool dual_on = dual.A2 != nullptr;
  const __amdgpu_buffer_rsrc_t ra2 =
      dual_on ? __builtin_amdgcn_make_buffer_rsrc((void*)dual.A2, (short)0, (int)dual.a2_bytes, 0x00020000) : ra;
  const __amdgpu_buffer_rsrc_t rb2 =
      dual_on ? __builtin_amdgcn_make_buffer_rsrc((void*)dual.B2, (short)0, (int)dual.b2_bytes, 0x00020000) : rb;
  const int lda2 = dual_on ? dual.lda2 : lda, ldb2 = dual_on ? dual.ldb2 : ldb;

  auto decode = [&](int lin, int& m0, int& n0, int& kb, int& ke, int& split, int& sel) {
    split = lin / nwg;
    const int wg = lin - split * nwg;
    const int per_group = group_m * tiles_n;
    const int gid = wg / per_group;
    const int first_m = gid * group_m;
    const int gsz = min(tiles_m - first_m, group_m);
    const int r = wg - gid * per_group;
    m0 = (first_m + r % gsz) * BM_;
    n0 = (r / gsz) * BN_;
    kb = split * k_per_split;
    ke = min(K, kb + k_per_split);
    sel = 0;
    if (kb >= dual.k_switch) {
      sel = 1;
      kb -= dual.k_switch;
      ke -= dual.k_switch;
    }
  };

  int it = xcd_remap(blockIdx.x, G);
  if (it >= total) return;
  int m0, n0, kb, ke, split, sel;
  decode(it, m0, n0, kb, ke, split, sel);
  issue_tile<AK, BM_, NWV>(sel ? ra2 : ra, smem, m0, kb, sel ? lda2 : lda, ke);
  issue_tile<BKM, BN_, NWV>(sel ? rb2 : rb, smem + A_BYTES, n0, kb, sel ? ldb2 : ldb, ke);
  int cur = 0;
  bool first = true;
  for (; it < total; it += G) {
    const bool has_next = it + G < total;
    int m0n = 0, n0n = 0, kbn = 0, ken = 0, splitn = 0, seln = 0;
    if (has_next) decode(it + G, m0n, n0n, kbn, ken, splitn, seln);
    const int nk = max(1, (ke - kb + 63) / 64);   // an empty K-split runs one all-zero step

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

    for (int t = 0; t < nk; ++t) {
      // The tile of step t is the youngest DMA batch but for the previous item's epilogue
      // stores (issued after it) at t == 0.
      if (t == 0 && !first) wait_vmcnt<STORES>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();  // tile t landed for all waves; the other stage is free
      const bool in_item = t + 1 < nk;
      const bool more = in_item || has_next;
      const int pm0 = in_item ? m0 : m0n, pn0 = in_item ? n0 : n0n;
      const int pk = in_item ? kb + (t + 1) * 64 : kbn, pke = in_item ? ke : ken;
      const int psel = in_item ? sel : seln;
      char* nst = smem + (cur ^ 1) * STAGE;
      const char* la = smem + cur * STAGE;
      const char* lb = la + A_BYTES;
      auto piece = [&](int q) {
        if (q < PA) issue_piece<AK, BM_, NWV>(psel ? ra2 : ra, nst, pm0, pk, psel ? lda2 : lda, pke, q);
        else issue_piece<BKM, BN_, NWV>(psel ? rb2 : rb, nst + A_BYTES, pn0, pk, psel ? ldb2 : ldb, pke, q - PA);
      };
      if constexpr (SCHED == 4) {
        bf16x8 fa[2][TM], fb[2][TN];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
#pragma unroll
          for (int j = 0; j < TN; ++j) fb[s][j] = frag2<BKM, BN_>(lb, wn * WN + 16 * j, 32 * s);
#pragma unroll
          for (int i = 0; i < TM; ++i) fa[s][i] = frag2<AK, BM_>(la, wm * WM + 16 * i, 32 * s);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[s][j], fa[s][i], acc[i][j], 0, 0, 0);
            if (s == 0 && more) {
#pragma unroll
              for (int q = 0; q < PIECES; ++q)
                if ((q * TM) / PIECES == i) piece(q);
            }
          }
          __builtin_amdgcn_s_setprio(0);
        }
      } else {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 fa[TM], fb[TN];
#pragma unroll
          for (int i = 0; i < TM; ++i) fa[i] = frag2<AK, BM_>(la, wm * WM + 16 * i, 32 * s);
#pragma unroll
          for (int j = 0; j < TN; ++j) fb[j] = frag2<BKM, BN_>(lb, wn * WN + 16 * j, 32 * s);
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < TM; ++i) {
#pragma unroll
            for (int j = 0; j < TN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
            if (s == 0 && more) {
#pragma unroll
              for (int q = 0; q < PIECES; ++q)
                if ((q * TM) / PIECES == i) piece(q);
            }
          }
          __builtin_amdgcn_s_setprio(0);
        }
      }
      cur ^= 1;
    }

    // Epilogue (as gemm2_k): lane holds C[m = .. + (l&15)][n = .. + 4g + r]; every wave issues
    // exactly TM*TN buffer stores, out-of-range lanes get an offset past num_records.
    const int g = l >> 4;
    const int wcol0 = n0 + wn * WN;
    char* cbase = reinterpret_cast<char*>(C) + (OUT == 1 ? (long long)split * slab_stride * 4 : 0);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void*)cbase, (short)0, (int)c_bytes, 0x00020000);
    const bool do_rope = (OUT == 0) && (WN % 64 == 0) && rope.cols > 0 && wcol0 < rope.cols;
    f32x4 bv[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = wcol0 + 16 * j + 4 * g;
      bv[j] = (OUT == 0 && bias && n < N) ? *reinterpret_cast<const f32x4*>(bias + n) : (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * WM + 16 * i + (l & 15);
      f32x4 v[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) v[j] = acc[i][j] + bv[j];
      if constexpr (OUT == 0 && WN % 64 == 0) {
        if (do_rope && m < M) {
          const float* tr = rope.tab + rope.pos[m] * 64;
#pragma unroll
          for (int hg = 0; hg < WN / 64; ++hg) {
            if (wcol0 + 64 * hg >= rope.cols) break;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const f32x4 cs = *reinterpret_cast<const f32x4*>(tr + 16 * j + 4 * g);
              const f32x4 sn = *reinterpret_cast<const f32x4*>(tr + 32 + 16 * j + 4 * g);
              const f32x4 x1 = v[4 * hg + j], x2 = v[4 * hg + j + 2];
              v[4 * hg + j] = x1 * cs - x2 * sn;
              v[4 * hg + j + 2] = x2 * cs + x1 * sn;
            }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = wcol0 + 16 * j + 4 * g;
        const bool ok = m < M && n < N;
        if (OUT == 0) {
          const unsigned off = ok ? (unsigned)(((long long)m * ldc + n) * 2) : kOOB;
          bf16x4 o = {(bf16)v[j][0], (bf16)v[j][1], (bf16)v[j][2], (bf16)v[j][3]};
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), rc, off, 0, 0);
        } else {
          const unsigned off = ok ? (unsigned)(((long long)m * ldc + n) * 4) : kOOB;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[j]), rc, off, 0, 0);
        }
      }
    }
    first = false;
    m0 = m0n;
    n0 = n0n;
    kb = kbn;
    ke = ken;
    split = splitn;
    sel = seln;
  }
}

// bf16 out[m*ldc + n] = sum_s slab[s][m*N + n] (+ bias[n]), fixed order; N % 4 == 0.
__global__ __launch_bounds__(256) void splitk_reduce_bf16_k(const float* __restrict__ slabs, bf16* __restrict__ out,
                                                            const float* __restrict__ bias, int M, int N, int ldc,
                                                            int S) {
  const long long n4 = (long long)M * N / 4;
  const long long stride = (long long)M * N;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const long long e = i * 4;
    const int m = (int)(e / N), n = (int)(e % N);
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < S; ++k) s += *reinterpret_cast<const f32x4*>(slabs + k * stride + e);
    if (bias) s += *reinterpret_cast<const f32x4*>(bias + n);
    bf16x4 o = {(bf16)s[0], (bf16)s[1], (bf16)s[2], (bf16)s[3]};
    *reinterpret_cast<bf16x4*>(out + (long long)m * ldc + n) = o;
  }
}

}  // namespace dpfs

using namespace dpfs;

static int tiles_of(int M, int N) { return ((M + BM - 1) / BM) * ((N + BN - 1) / BN); }
static int tiles2(int M, int N, int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); }

static unsigned span_bytes(long long rows, long long ld, long long cols) {
  // bytes from the base to the end of the last row of a (rows x cols, stride ld) bf16 view
  const long long b = rows > 0 ? ((rows - 1) * ld + cols) * 2 : 0;
  return (unsigned)b;
}

// DMA-issue / fragment-read schedule of the 256x256 tile (gemm2_k SCHED), per layout, from
// tools/gemm_probe.py sweeps on MI355X (profiles/r1_gemm_sched_sweep.log): NT 2 (+7 %),
// NN and TN 4 (+16..30 % over issuing every DMA piece right after the barrier).
static int g_v2_sched = -1;  // -1 = per-layout default
extern "C" void dpfs_gemm_v2_sched(int v) { g_v2_sched = v; }
template <bool AK, bool BKM>
static int v2_sched() {
  if (g_v2_sched >= 0) return g_v2_sched;
  return (AK && BKM) ? 2 : 4;
}

// v2 configurations: 0 = 256x256 / 2-stage (128 KiB LDS), 1 = 256x128 / 3-stage (144 KiB).
template <bool AK, bool BKM, int OUT>
static void launch2(int cfg, const void* A, const void* B, void* C, const float* bias, int M, int N, int K, int lda,
                    int ldb, int ldc, int splits, int kps, long long slab, unsigned ab, unsigned bb, hipStream_t s,
                    RopeArgs rope = RopeArgs{nullptr, nullptr, 0}) {
  if (cfg == 0) {
    const dim3 grid(tiles2(M, N, 256, 256), splits);
    const int sched = v2_sched<AK, BKM>();
    if (sched == 1)
      gemm2_k<256, 256, 2, 2, AK, BKM, OUT, 1><<<grid, 512, 0, s>>>((const bf16*)A, (const bf16*)B, C, bias, M, N, K,
                                                                  lda, ldb, ldc, kps, slab, ab, bb, rope);
    else if (sched == 2)
      gemm2_k<256, 256, 2, 2, AK, BKM, OUT, 2><<<grid, 512, 0, s>>>((const bf16*)A, (const bf16*)B, C, bias, M, N, K,
                                                                  lda, ldb, ldc, kps, slab, ab, bb, rope);
    else if (sched == 3)
      gemm2_k<256, 256, 2, 2, AK, BKM, OUT, 3><<<grid, 512, 0, s>>>((const bf16*)A, (const bf16*)B, C, bias, M, N, K,
                                                                  lda, ldb, ldc, kps, slab, ab, bb, rope);
    else if (sched == 4)
      gemm2_k<256, 256, 2, 2, AK, BKM, OUT, 4><<<grid, 512, 0, s>>>((const bf16*)A, (const bf16*)B, C, bias, M, N, K,
                                                                  lda, ldb, ldc, kps, slab, ab, bb, rope);
    else
      gemm2_k<256, 256, 2, 2, AK, BKM, OUT, 0><<<grid, 512, 0, s>>>((const bf16*)A, (const bf16*)B, C, bias, M, N, K,
                                                                  lda, ldb, ldc, kps, slab, ab, bb, rope);
  } else {
    const dim3 grid(tiles2(M, N, 256, 128), splits);
    if (v2_sched<AK, BKM>() == 4)
      gemm2_k<256, 128, 4, 3, AK, BKM, OUT, 4><<<grid, 512, 0, s>>>((const bf16*)A, (const bf16*)B, C, bias, M, N, K,
                                                                  lda, ldb, ldc, kps, slab, ab, bb, rope);
    else
      gemm2_k<256, 128, 4, 3, AK, BKM, OUT, 2><<<grid, 512, 0, s>>>((const bf16*)A, (const bf16*)B, C, bias, M, N, K,
                                                                  lda, ldb, ldc, kps, slab, ab, bb, rope);
  }
}

// Persistent v3 launch (gemmp_k): grid = min(items, CUs) (one 512-thread workgroup per CU:
// 128 KiB LDS), NSTAGE 2 for both tile shapes.  Returns false when an operand / output span
// does not fit the 32-bit buffer descriptors (then the caller runs v2).
static int g_group_m = 4;
extern "C" void dpfs_gemm_group_m(int g) { g_group_m = g > 0 ? g : 4; }
static int cu_count() {
  static int n[16] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 16) dev = 0;
  if (n[dev] == 0) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    n[dev] = c;
  }
  return n[dev];
}
template <bool AK, bool BKM, int OUT>
static bool launchp(int cfg, const void* A, const void* B, void* C, const float* bias, int M, int N, int K, int lda,
                    int ldb, int ldc, int splits, int kps, long long slab, unsigned ab, unsigned bb, hipStream_t s,
                    RopeArgs rope = RopeArgs{nullptr, nullptr, 0}, Dual dual = kNoDual) {
  const long long cspan = M > 0 ? ((long long)(M - 1) * ldc + N) * (OUT == 1 ? 4 : 2) : 0;
  if (cspan >= (1ll << 32) - 16) return false;
  const int bm = 256, bn = cfg == 0 ? 256 : 128;
  const long long items = (long long)tiles2(M, N, bm, bn) * splits;
  if (items <= 0 || items >= (1ll << 31)) return false;
  const int grid = (int)std::min<long long>(items, cu_count());
  const int sched = v2_sched<AK, BKM>() == 4 ? 4 : 2;
  const unsigned cb = (unsigned)cspan;
#define GEMMP_LAUNCH(BN_, WM_, SC_)                                                                                    \
  gemmp_k<256, BN_, WM_, AK, BKM, OUT, SC_><<<grid, 512, 0, s>>>((const bf16*)A, (const bf16*)B, C, bias, M, N, K,  \
                                                                lda, ldb, ldc, kps, splits, slab, ab, bb, cb, rope, \
                                                                g_group_m, dual)
  if (cfg == 0) {
    if (sched == 4) GEMMP_LAUNCH(256, 2, 4);
    else GEMMP_LAUNCH(256, 2, 2);
  } else {
    if (sched == 4) GEMMP_LAUNCH(128, 4, 4);
    else GEMMP_LAUNCH(128, 4, 2);
  }
#undef GEMMP_LAUNCH
  return true;
}

static int g_force_cfg = -1;     // -1 auto, 0 = 256x256, 1 = 256x128 (tuning / A-B runs)
static int g_force_splits = 0;   // 0 auto
extern "C" void dpfs_gemm_force(int cfg, int splits) {
  g_force_cfg = cfg;
  g_force_splits = splits;
}

// Tile choice (measured with tools/tune_gemm.py, see profiles/): 256x256 unless the
// 256x128 tile wastes less of a ragged N (e.g. N = 384 at TP=8).
static int pick_cfg(int M, int N, int splits) {
  if (g_force_cfg >= 0) return g_force_cfg;
  const int w0 = ((N + 255) / 256) * 256 - N, w1 = ((N + 127) / 128) * 128 - N;
  return (w1 < w0 && w0 * 10 > N) ? 1 : 0;  // only when the 256-wide tile wastes > 10% of N
}

// K-splits: grow while the grid stays <= ~1300 blocks (~5 waves of 256 CUs) and each split
// keeps >= 4096 of K (fp32 slab round trip < ~10% of the split's MFMA time).
static int v2_splits(int M, int N, int K, int cfg) {
  const int tiles = cfg == 0 ? tiles2(M, N, 256, 256) : tiles2(M, N, 256, 128);
  int s = 1;
  while (s < 64 && tiles * s * 2 <= 1300 && K / (s * 2) >= 4096) s *= 2;
  return s;
}

// Split-K for bf16-output GEMMs whose tile grid under-fills 256 CUs while K is long
// (e.g. the lm_head dgrad: N = d_model, K = vocab shard).
static int bf16_splits(int M, int N, int K) {
  if (g_force_splits > 0) return g_force_splits;
  return v2_splits(M, N, K, pick_cfg(M, N, 1));
}

static int g_gemm_impl = 3;  // 3 = v3 persistent (default), 2 = v2 one tile per workgroup, 1 = v1
extern "C" void dpfs_gemm_set_impl(int v) { g_gemm_impl = v; }

static thread_local float* g_ws = nullptr;  // split-K workspace for bf16 outputs (set by host)
static thread_local long long g_ws_floats = 0;
extern "C" void dpfs_gemm_set_workspace(float* ws, long long n) {
  g_ws = ws;
  g_ws_floats = n;
}
extern "C" void dpfs_rope(int dtype, void* qkv, const int64_t* pos, const float* table, int M, int ld, int n_heads,
                          int hd, int inverse, hipStream_t s);
static void dpfs_rope_after_gemm(void* C, RopeArgs r, int M, int ldc, hipStream_t s) {
  dpfs_rope(1, C, r.pos, r.tab, M, ldc, r.cols / r.hd, r.hd, 0, s);
}

// v4 (csrc/kernels/gemm4.hip: one wave per SIMD, 128 x 128 per wave).  Bit mask of the
// layouts it carries: 1 = NT, 2 = NN, 4 = TN (fp32 split-K).  Where the launcher declines a
// shape (32-bit spans, alignment) the v3 kernel runs.
extern "C" bool dpfs_gemm4_launch(int layout, int out_f32, const void* A, const void* B, void* C, const float* bias,
                                  int M, int N, int K, int lda, int ldb, int ldc, int kps, int splits,
                                  long long slab_stride, unsigned a_bytes, unsigned b_bytes, const int64_t* rope_pos,
                                  const float* rope_tab, int rope_cols, int rope_hd, const void* A2, const void* B2,
                                  int k_switch, int lda2, int ldb2, unsigned a2_bytes, unsigned b2_bytes,
                                  int bn_force, hipStream_t s);

// Per-call kernel variant (an argument of every GEMM entry point, never process state):
//   0 = v4 with its per-shape tile width (the default for every layout),
//   1 / 2 = v4 with the 256 / 192 tile width forced (non-split bf16 NT / NN),
//   3 = the v3 kernel (8 waves, 128 x 64 per wave);
//   + 4 (variants 4 / 5 / 6): the v4 bf16 output written with non-temporal (streaming)
//   stores, so the output does not displace the operands in L2 (plain NT / NN only).
// Where the v4 launcher declines a shape (32-bit spans, alignment) the v3 kernel runs.
static bool use_v4(int variant) { return g_gemm_impl >= 3 && (variant & 3) != 3; }
static int v4_bn(int variant) {
  const int w = variant & 3;
  return (w == 1 ? 256 : (w == 2 ? 192 : 0)) | ((variant & 4) ? 0x100 : 0) | ((variant & 8) ? 0x200 : 0);
}
extern "C" void dpfs_gemm4_set_sk_ws(float* p, long long n);
extern "C" long long dpfs_gemm4_sk_ws(int M, int N, int K);

extern "C" long long dpfs_gemm_bf16_ws(int M, int N, int K) {
  const int S = bf16_splits(M, N, K);
  return S > 1 ? (long long)S * M * N : 0;
}

template <bool BKM>
static void bf16_gemm(const void* A, const void* B, void* C, const float* bias, int M, int N, int K, int lda, int ldb,
                      int ldc, unsigned ab, unsigned bb, int variant, hipStream_t s,
                      RopeArgs rope = RopeArgs{nullptr, nullptr, 0}) {
  const bool v4 = use_v4(variant);
  // stream-K requested where it applies: it replaces the split-K slabs (a long-K shape whose
  // 256 x 256 tiles are 1.5 per CU, e.g. the lm_head data gradient)
  const bool sk = v4 && (variant & 8) && rope.cols == 0 && dpfs_gemm4_sk_ws(M, N, K) > 0;
  const int S = sk ? 1 : bf16_splits(M, N, K);
  const int lay = BKM ? 0 : 1;
  if (S > 1 && g_ws && g_ws_floats >= (long long)S * M * N) {
    int kps = (K + S - 1) / S;
    kps = ((kps + BKK - 1) / BKK) * BKK;
    const bool done4 = v4 && dpfs_gemm4_launch(lay, 1, A, B, g_ws, nullptr, M, N, K, lda, ldb, N, kps, S,
                                               (long long)M * N, ab, bb, nullptr, nullptr, 0, 64, nullptr, nullptr, 0,
                                               0, 0, 0u, 0u, 0, s);
    if (!done4 && (g_gemm_impl != 3 || !launchp<true, BKM, 1>(pick_cfg(M, N, S), A, B, g_ws, nullptr, M, N, K, lda,
                                                               ldb, N, S, kps, (long long)M * N, ab, bb, s)))
      launch2<true, BKM, 1>(pick_cfg(M, N, S), A, B, g_ws, nullptr, M, N, K, lda, ldb, N, S, kps, (long long)M * N, ab,
                            bb, s);
    long long g = ((long long)M * N / 4 + 255) / 256;
    if (g > 4096) g = 4096;
    splitk_reduce_bf16_k<<<(int)g, 256, 0, s>>>(g_ws, (bf16*)C, bias, M, N, ldc, S);
    if (rope.cols > 0) dpfs_rope_after_gemm(C, rope, M, ldc, s);
    return;
  }
  if (variant & 8) dpfs_gemm4_set_sk_ws(g_ws, g_ws_floats);   // (stream-K: its partials / flags)
  const bool done4 = v4 && dpfs_gemm4_launch(lay, 0, A, B, C, bias, M, N, K, lda, ldb, ldc, ((K + 31) / 32) * 32, 1, 0,
                                             ab, bb, rope.pos, rope.tab, rope.cols, rope.hd, nullptr, nullptr, 0, 0, 0,
                                             0u, 0u, v4_bn(variant), s);
  if (variant & 8) dpfs_gemm4_set_sk_ws(nullptr, 0);
  if (done4) return;
  if (rope.cols > 0 && rope.hd != 64) {   // v3's epilogue rotates 64-wide heads only
    bf16_gemm<BKM>(A, B, C, bias, M, N, K, lda, ldb, ldc, ab, bb, variant, s);
    dpfs_rope_after_gemm(C, rope, M, ldc, s);
    return;
  }
  if (g_gemm_impl == 3 && launchp<true, BKM, 0>(pick_cfg(M, N, 1), A, B, C, bias, M, N, K, lda, ldb, ldc, 1, K, 0, ab,
                                                bb, s, rope))
    return;
  launch2<true, BKM, 0>(pick_cfg(M, N, 1), A, B, C, bias, M, N, K, lda, ldb, ldc, 1, K, 0, ab, bb, s, rope);
}

// Whether dpfs_gemm_nt_rope fuses the rotation into the GEMM epilogue (hd 64; otherwise it
// runs the separate RoPE kernel after the GEMM — same result).
extern "C" int dpfs_gemm_rope_fusable(int M, int N, int K, int hd, int variant) {
  if (g_gemm_impl == 1) return 0;
  if (hd == 64) return N % 64 == 0;
  return hd == 128 && use_v4(variant) && N % 128 == 0;
}

extern "C" void dpfs_gemm_nt_rope(const void* A, const void* B, void* C, const float* bias, int M, int N, int K,
                                  int lda, int ldb, int ldc, const int64_t* pos, const float* tab, int rope_cols,
                                  int rope_hd, int variant, hipStream_t s) {
  bf16_gemm<true>(A, B, C, bias, M, N, K, lda, ldb, ldc, span_bytes(M, lda, K), span_bytes(N, ldb, K), variant, s,
                  RopeArgs{pos, tab, rope_cols, rope_hd});
}

// NT: C[M,N] bf16 = A[M,K] B[N,K]^T (+ bias)
extern "C" void dpfs_gemm_nt(const void* A, const void* B, void* C, const float* bias, int M, int N, int K, int lda,
                             int ldb, int ldc, int variant, hipStream_t s) {
  if (g_gemm_impl == 1) {
    gemm_k<true, true, 0><<<dim3(tiles_of(M, N), 1), 256, 0, s>>>((const bf16*)A, (const bf16*)B, C, bias, M, N, K,
                                                                 lda, ldb, ldc, K, 0);
    return;
  }
  bf16_gemm<true>(A, B, C, bias, M, N, K, lda, ldb, ldc, span_bytes(M, lda, K), span_bytes(N, ldb, K), variant, s);
}

// NN: C[M,N] bf16 = A[M,K] B[K,N]
extern "C" void dpfs_gemm_nn(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                             int variant, hipStream_t s) {
  if (g_gemm_impl == 1) {
    gemm_k<true, false, 0><<<dim3(tiles_of(M, N), 1), 256, 0, s>>>((const bf16*)A, (const bf16*)B, C, nullptr, M, N,
                                                                  K, lda, ldb, ldc, K, 0);
    return;
  }
  bf16_gemm<false>(A, B, C, nullptr, M, N, K, lda, ldb, ldc, span_bytes(M, lda, K), span_bytes(K, ldb, N), variant, s);
}

// TN (wgrad) plan.  Outputs are small (weight shards) and K = tokens is long, so the K-split
// count S sets the grid.  v2 256x256: S (K/S >= 512) minimising a makespan model
// calibrated on MI355X sweeps (profiles/r1_gemm_tn_sweep.log, within ~10 % on every TP1-8
// GPT-2 wgrad shape):  ceil(tiles*S / 256 CUs) * ceil(K/S / 64) * 1.95 us   (one 256x256x64
// K-step per CU)  +  S*M*N*8 B / 4 TB/s  (fp32 slabs written + reduced).  The 128x128 v1
// kernel when the 256-granular tiles waste > 30 % of the output (e.g. 576- or 384-row
// shards at TP 4 / 8).
static int tn_v2_splits(int M, int N, int K) {
  const long long tiles = tiles2(M, N, 256, 256);
  int best = 1;
  double best_t = 1e300;
  // Every split count, not only powers of 2: the lm_head wgrad (591 tiles = 2.3 rounds of 256
  // CUs) runs best at S = 3 (7 full rounds): 2.44 vs 2.58 ms at S = 2 (tools/tn_lmhead_probe.py).
  for (int S = 1; S <= 64; ++S) {
    if (S > 1 && K / S < 512) break;
    const long long kps = ((K + S - 1) / S + 63) / 64;
    const long long rounds = (tiles * S + 255) / 256;
    const double t = (double)rounds * kps * 1.95 + (S > 1 ? (double)S * M * N * 8.0 / 4.0e6 : 0.0);
    if (t < best_t * 0.97) {
      best_t = t;
      best = S;
    }
  }
  return best;
}

// Small outputs (fewer than 256 tiles of 256x256: every TP-sharded wgrad at TP 4-8, e.g.
// 384 x 768 or 768 x 128 at TP 8) cannot fill the chip without a K-split, and power-of-2
// splits leave ragged rounds (6 tiles x 64 = 384 blocks = 1.5 rounds).  Search every split
// 1..64 and both tile shapes with the makespan model (256x128 K-step ~1.5 us); measured on
// the TP 8 shapes (tools/tn_split_sweep.py): 384x768 0.182 -> 0.140 ms (6 tiles x 42 splits),
// 768x128 0.081 -> 0.069 ms (256x128 tiles, 64 splits).
static int tn_small_plan(int M, int N, int K, int* cfg) {
  double best_t = 1e300;
  int best_s = 1;
  *cfg = 0;
  for (int c = 0; c < 2; ++c) {
    const long long tiles = c == 0 ? tiles2(M, N, 256, 256) : tiles2(M, N, 256, 128);
    const double step = c == 0 ? 1.95 : 1.5;
    for (int S = 1; S <= 64; ++S) {
      if (S > 1 && K / S < 512) break;
      const long long kps = ((K + S - 1) / S + 63) / 64;
      const long long rounds = (tiles * S + 255) / 256;
      const double t = (double)rounds * kps * step + (S > 1 ? (double)S * M * N * 8.0 / 4.0e6 : 0.0);
      if (t < best_t * 0.97) {
        best_t = t;
        best_s = S;
        *cfg = c;
      }
    }
  }
  return best_s;
}

static bool tn_use_v1(int M, int N, int K) { return g_gemm_impl == 1; }

// (tile config, K-splits) of a TN GEMM.
static int tn_plan(int M, int N, int K, int* cfg) {
  *cfg = g_force_cfg >= 0 ? g_force_cfg : 0;
  if (tn_use_v1(M, N, K)) {
    const int tiles = tiles_of(M, N);
    int s = 1;
    while (tiles * s < 256 && (K / (s * 2)) >= 8 * BKK && s < 64) s *= 2;
    return s;
  }
  if (g_force_splits > 0) return g_force_splits;
  if (g_force_cfg < 0 && tiles2(M, N, 256, 256) < 256) return tn_small_plan(M, N, K, cfg);
  return tn_v2_splits(M, N, K);
}

extern "C" int dpfs_gemm_tn_splits(int M, int N, int K) {
  int cfg;
  return tn_plan(M, N, K, &cfg);
}

// Floats of slab workspace dpfs_gemm_tn needs (0: none).
extern "C" long long dpfs_gemm_tn_ws(int M, int N, int K, int accumulate) {
  const int S = dpfs_gemm_tn_splits(M, N, K);
  return (S > 1 || accumulate) ? (long long)S * M * N : 0;
}

// TN: C[M,N] fp32 (+)= A[K,M]^T B[K,N].  ws: splits*M*N floats when splits > 1 or accumulate.
extern "C" void dpfs_gemm_tn(const void* A, const void* B, float* C, float* ws, int M, int N, int K, int lda, int ldb,
                             int accumulate, int variant, hipStream_t s) {
  const long long n = (long long)M * N;
  int cfg;
  const int S = tn_plan(M, N, K, &cfg);
  int kps = (K + S - 1) / S;
  kps = ((kps + BKK - 1) / BKK) * BKK;
  const bool direct = (S == 1 && !accumulate);
  float* dst = direct ? C : ws;
  if (use_v4(variant)) {
    const int S4 = g_force_splits > 0 ? g_force_splits : tn_v2_splits(M, N, K);
    if (S4 == S || (S4 < S)) {   // v4 plans with 256 x 256 tiles; its split count never needs more slabs
      int kps4 = (K + S4 - 1) / S4;
      kps4 = ((kps4 + BKK - 1) / BKK) * BKK;
      const bool direct4 = (S4 == 1 && !accumulate);
      if (dpfs_gemm4_launch(2, 1, A, B, direct4 ? C : ws, nullptr, M, N, K, lda, ldb, N, direct4 ? ((K + 31) / 32) * 32 : kps4,
                            S4, direct4 ? 0 : n, span_bytes(K, lda, M), span_bytes(K, ldb, N), nullptr, nullptr, 0, 64,
                            nullptr, nullptr, 0, 0, 0, 0u, 0u, 0, s)) {
        if (direct4) return;
        long long g = (n / 4 + 255) / 256;
        if (g > 4096) g = 4096;
        splitk_reduce_k<<<(int)g, 256, 0, s>>>(ws, C, n, S4, accumulate);
        return;
      }
    }
  }
  if (tn_use_v1(M, N, K)) {
    gemm_k<false, false, 1><<<dim3(tiles_of(M, N), S), 256, 0, s>>>((const bf16*)A, (const bf16*)B, dst, nullptr, M,
                                                                   N, K, lda, ldb, N, direct ? K : kps,
                                                                   direct ? 0 : n);
  } else if (g_gemm_impl != 3 ||
             !launchp<false, false, 1>(cfg, A, B, dst, nullptr, M, N, K, lda, ldb, N, S, direct ? K : kps,
                                       direct ? 0 : n, span_bytes(K, lda, M), span_bytes(K, ldb, N), s)) {
    launch2<false, false, 1>(cfg, A, B, dst, nullptr, M, N, K, lda, ldb, N, S, direct ? K : kps,
                             direct ? 0 : n, span_bytes(K, lda, M), span_bytes(K, ldb, N), s);
  }
  if (direct) return;
  long long g = (n / 4 + 255) / 256;
  if (g > 4096) g = 4096;
  splitk_reduce_k<<<(int)g, 256, 0, s>>>(ws, C, n, S, accumulate);
}

// TN with the reduction dim split over two buffer pairs (a chunked step's two ping-pong
// chunks): C[M,N] fp32 (+)= A0[K0,M]^T B0[K0,N] + A1[K1,M]^T B1[K1,N] as ONE persistent
// split-K launch and ONE slab reduction, planned as dpfs_gemm_tn over K0 + K1 (so the same
// tile / split counts as one tall GEMM; two separate calls pay two reductions and two
// under-filled grids).  ws: dpfs_gemm_tn2_ws floats.  Returns 0 (nothing launched) when no
// K-split length divides K0 (a split must not straddle the two buffers).
static int tn2_plan(int M, int N, int K0, int K1, int* cfg_out, int* kps_out) {
  if (g_gemm_impl != 3 || K0 <= 0 || K1 <= 0) return 0;
  const int K = K0 + K1;
  int cfg;
  (void)tn_plan(M, N, K, &cfg);
  // K-split length: a divisor K0 / j (multiple of 64) so no split straddles the buffers,
  // chosen with the makespan model of tn_small_plan over the whole K0 + K1.
  const long long tiles = cfg == 0 ? tiles2(M, N, 256, 256) : tiles2(M, N, 256, 128);
  const double step = cfg == 0 ? 1.95 : 1.5;
  int kps = 0, S = 0;
  double best = 1e300;
  for (int j = 1; j <= 64; ++j) {
    if (K0 % j) continue;
    const int kp = K0 / j;
    if (kp % BKK || kp < 512) continue;
    const int Sj = (K + kp - 1) / kp;
    if (Sj < 2 || Sj > 64) continue;
    const double t = (double)((tiles * Sj + 255) / 256) * (kp / 64) * step + (double)Sj * M * N * 8.0 / 4.0e6;
    if (t < best * 0.97) {
      best = t;
      kps = kp;
      S = Sj;
    }
  }
  *cfg_out = cfg;
  *kps_out = kps;
  return S;
}

extern "C" long long dpfs_gemm_tn2_ws(int M, int N, int K0, int K1) {
  int cfg, kps;
  const int S = tn2_plan(M, N, K0, K1, &cfg, &kps);
  return (long long)S * M * N;
}

extern "C" int dpfs_gemm_tn2(const void* A0, const void* B0, const void* A1, const void* B1, float* C, float* ws,
                             int M, int N, int K0, int K1, int lda0, int ldb0, int lda1, int ldb1, int accumulate,
                             int variant, hipStream_t s) {
  int cfg, kps;
  const int S = tn2_plan(M, N, K0, K1, &cfg, &kps);
  if (S == 0) return 0;
  const int K = K0 + K1;
  const long long n = (long long)M * N;
  const Dual d = {(const bf16*)A1, (const bf16*)B1, K0, lda1, ldb1, span_bytes(K1, lda1, M), span_bytes(K1, ldb1, N)};
  const bool done4 = use_v4(variant) &&
                     dpfs_gemm4_launch(2, 1, A0, B0, ws, nullptr, M, N, K, lda0, ldb0, N, kps, S, n,
                                       span_bytes(K0, lda0, M), span_bytes(K0, ldb0, N), nullptr, nullptr, 0, 64, A1,
                                       B1, K0, lda1, ldb1, d.a2_bytes, d.b2_bytes, 0, s);
  if (!done4 && !launchp<false, false, 1>(cfg, A0, B0, ws, nullptr, M, N, K, lda0, ldb0, N, S, kps, n, span_bytes(K0, lda0, M),
                                span_bytes(K0, ldb0, N), s, RopeArgs{nullptr, nullptr, 0}, d))
    return 0;
  long long g = (n / 4 + 255) / 256;
  if (g > 4096) g = 4096;
  splitk_reduce_k<<<(int)g, 256, 0, s>>>(ws, C, n, S, accumulate);
  return 1;
}
