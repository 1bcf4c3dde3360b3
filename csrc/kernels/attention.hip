// Causal flash attention (forward + backward) for gfx950, bf16 in / fp32 accumulate.
//
// Replaces the reference's materialised attention (models/model.py:73-77: QK^T, a
// (B,1,T,T) triu mask built every layer and step, masked_fill, softmax, P.V and their
// autograd backward) with O(T)-memory kernels; the log-sum-exp per query
// row is the only saved statistic.
//
// Layout: q/k/v/do are (B, T, H, hd) views with token stride `ld` (the packed QKV GEMM
// output: ld = 3*H*hd), o/dq/dk/dv likewise with their own strides; lse/delta are (B, H, T).
//
// MFMA orientation (v_mfma_f32_16x16x32_bf16; C/D map col = lane&15, row = 4*(lane>>4)+j):
//  * forward and dQ compute the TRANSPOSED score tile S^T = K Q^T, so each lane owns one
//    query column: the row max / row sum / rescale of the online softmax are lane-local
//    (plus one xor-16/32 butterfly), and P^T in registers is directly the B operand of
//    O^T = V^T P^T (k-slot permutation shared with the V^T operand, which is fetched with
//    the CDNA4 transpose read ds_read_b64_tr_b16) — P never touches LDS.
//  * dK/dV compute S = Q K^T with the block's keys held in registers; P^T/dS^T are then
//    the A operands of dV = P^T dO and dK = dS^T Q without data movement.
//  * backward = a dQ kernel (one block per 128 queries; it also computes and stores
//    delta = rowsum(dO*O)) then a dK/dV kernel (one block per 64 keys): no float atomics,
//    bitwise deterministic.
//  * every LDS tile [rows][hd] uses one XOR swizzle that is conflict-free both for row
//    reads (ds_read_b128) and for transposed reads (ds_read_b64_tr_b16).
//  * causal: key tiles above the diagonal are never visited; heaviest q-blocks launch first.
#include "common.h"
#include "attn_common.h"

#include <algorithm>

namespace dpfs {

// Global -> registers -> swizzled LDS tile of R rows x HD (rows >= nvalid are zero).
template <int HD, int R, int NT = 256>
struct Stage {
  static constexpr int CPR = HD / 8;            // chunks per row
  static constexpr int NCH = R * CPR;          // chunks per tile
  static constexpr int NC = (NCH + NT - 1) / NT;  // chunks per thread (last round may be partial)
  u32x4 reg[NC];
  __device__ __forceinline__ void load(const bf16* base, long long ld, int nvalid) {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = threadIdx.x + NT * i;
      const int r = c / CPR, ch = c % CPR;
      u32x4 v = {0u, 0u, 0u, 0u};
      if ((NCH % NT == 0 || c < NCH) && r < nvalid) v = *reinterpret_cast<const u32x4*>(base + r * ld + ch * 8);
      reg[i] = v;
    }
  }
  __device__ __forceinline__ void store(char* lds) const {
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = threadIdx.x + NT * i;
      if (NCH % NT == 0 || c < NCH) *reinterpret_cast<u32x4*>(lds + sw_off<HD>(c / CPR, c % CPR)) = reg[i];
    }
  }
};

// =============================================================================== forward ==
// Block: NW waves x QW queries of one (b, h); K/V tiles of 64 keys, double buffered in LDS
// (measured at hd 64: 4 waves x 32 queries beats 8 waves, 16-query waves (occupancy 4) and
// issuing the next tile's loads after QK^T; profiles/r1_v4_attn_fwd_pmc.txt).
template <int HD, int NW = 4, int QW = 32>
__global__ __launch_bounds__(64 * NW, (HD > 64 ? 1 : 2)) void attn_fwd_k(const bf16* __restrict__ Q, const bf16* __restrict__ K,
                                                     const bf16* __restrict__ V, bf16* __restrict__ O,
                                                     float* __restrict__ LSE, int T, int H, long long ldq,
                                                     long long ldk, long long ldv, long long ldo, float scale,
                                                     int causal) {
  constexpr int QC = QW / 16;  // 16-query column tiles per wave
  constexpr int BQ = QW * NW, BKV = 64, KT = HD / 32, DT = HD / 16;
  constexpr int TILE = BKV * HD * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE];
  const int nqb = (T + BQ - 1) / BQ;
  // XCD-aware order: the blocks of one (b, h) -- which share its K / V -- run on one XCD
  // (one L2); within a head the heaviest query blocks still go first.
  const int xl = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
  const int qb = nqb - 1 - xl % gridDim.x;  // heaviest first
  const int bh = xl / gridDim.x, b = bh / H, h = bh % H;
  const int q0 = qb * BQ;
  const int wave = threadIdx.x >> 6, l = lane_id(), g = l >> 4;
  const int wq0 = q0 + wave * QW;
  const float c2 = scale * kLog2e;

  const bf16* qbase = Q + (long long)b * T * ldq + (long long)h * HD;
  const bf16* kbase = K + (long long)b * T * ldk + (long long)h * HD;
  const bf16* vbase = V + (long long)b * T * ldv + (long long)h * HD;

  // Q^T operand in registers: lane holds Q[wq0 + 16c + (l&15)][32kk + 8g + j].
  bf16x8 qf[QC][KT];
#pragma unroll
  for (int c = 0; c < QC; ++c) {
    const int qi = wq0 + 16 * c + (l & 15);
#pragma unroll
    for (int kk = 0; kk < KT; ++kk) {
      bf16x8 v = {};
      if (qi < T) v = *reinterpret_cast<const bf16x8*>(qbase + (long long)qi * ldq + 32 * kk + 8 * g);
      qf[c][kk] = v;
    }
  }

  f32x4 o[QC][DT];
#pragma unroll
  for (int c = 0; c < QC; ++c)
#pragma unroll
    for (int d = 0; d < DT; ++d) o[c][d] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float m[QC], lsum[QC];
#pragma unroll
  for (int c = 0; c < QC; ++c) {
    m[c] = -INFINITY;
    lsum[c] = 0.f;
  }

  const int kv_end = causal ? min(T, q0 + BQ) : T;
  const int nkv = (kv_end + BKV - 1) / BKV;
  Stage<HD, BKV, 64 * NW> sk, sv;
  sk.load(kbase, ldk, min(BKV, T));
  sv.load(vbase, ldv, min(BKV, T));
  sk.store(smem);
  sv.store(smem + TILE);
  __syncthreads();

  for (int t = 0; t < nkv; ++t) {
    const int cur = t & 1;
    const char* lk = smem + cur * 2 * TILE;
    const char* lv = lk + TILE;
    const int kv0 = t * BKV;
    const bool more = t + 1 < nkv;
    if (more) {
      const int n0 = kv0 + BKV;
      sk.load(kbase + (long long)n0 * ldk, ldk, min(BKV, T - n0));
      sv.load(vbase + (long long)n0 * ldv, ldv, min(BKV, T - n0));
    }
    const bool wave_active = !causal || kv0 <= wq0 + QW - 1;
    if (wave_active) {
      // S^T tiles: s[i][c] = K[kv0+16i..][:] . Q[16c..][:]^T
      f32x4 s[4][QC];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int c = 0; c < QC; ++c) s[i][c] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KT; ++kk) {
          const bf16x8 kf = row_frag<HD>(lk, 16 * i, 32 * kk);
#pragma unroll
          for (int c = 0; c < QC; ++c) s[i][c] = MFMA(kf, qf[c][kk], s[i][c]);
        }
      }
      // Online softmax per query column (lane-local + butterfly over the 4 lane groups).
      // The causal / tail mask is evaluated only on tiles that need it (wave-uniform), the
      // 1/sqrt(hd)*log2(e) scale is folded into the exp2 argument with one FMA, and every
      // visited tile has >= 1 valid key per query (key kv0 <= wq0), so no -inf guards.
      const bool need_mask = __builtin_amdgcn_readfirstlane(
          (int)((causal && kv0 + BKV - 1 > wq0) || (kv0 + BKV > T)));
#pragma unroll
      for (int c = 0; c < QC; ++c) {
        const int qi = wq0 + 16 * c + (l & 15);
        if (need_mask) {   // wave-uniform; branch-free selects
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int ki = kv0 + 16 * i + 4 * g + j;
              const bool z = (ki >= T) | (causal & (ki > qi));
              s[i][c][j] = z ? -INFINITY : s[i][c][j];
            }
        }
        float mx = s[0][c][0];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) mx = fmaxf(mx, s[i][c][j]);
        mx = group4_max(mx);
        // Deferred rescale: the running max m moves only when this tile's max exceeds it by
        // more than kDefer (log2 units).  Otherwise p = exp2(s c2 - m) <= 2^kDefer, exact in
        // fp32 and representable in bf16, and the final 1/l normalisation (and lse = m +
        // log2 l) is unchanged; the alpha exp and the O / l rescale run only on the (wave-
        // uniform) tiles where some column's max grew that much — rarely after the first.
        constexpr float kDefer = 8.f;
        const bool grow = mx * c2 > m[c] + kDefer;
        if (__builtin_amdgcn_ballot_w64(grow) != 0) {
          const float mnew = grow ? mx * c2 : m[c];
          const float alpha = __builtin_amdgcn_exp2f(m[c] - mnew);
          m[c] = mnew;
          lsum[c] *= alpha;
#pragma unroll
          for (int d = 0; d < DT; ++d) o[c][d] *= alpha;
        }
        const float mc = m[c];
        float ps = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float pv = __builtin_amdgcn_exp2f(fmaf(s[i][c][j], c2, -mc));
            s[i][c][j] = pv;
            ps += pv;
          }
        lsum[c] += ps;
      }
      // O^T[d][q] += V^T[d][k] P^T[k][q]
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 pc[QC];
#pragma unroll
        for (int c = 0; c < QC; ++c) pc[c] = pack_pt(s[2 * ks][c], s[2 * ks + 1][c]);
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          const bf16x8 vf = tr_frag<HD>(lv, 32 * ks, 16 * d);
#pragma unroll
          for (int c = 0; c < QC; ++c) o[c][d] = MFMA(vf, pc[c], o[c][d]);
        }
      }
    }
    if (more) {
      char* nk = smem + (cur ^ 1) * 2 * TILE;
      sk.store(nk);
      sv.store(nk + TILE);
    }
    __syncthreads();
  }

  // Epilogue: O[q][d] = O^T[d][q] / l ; lse = (m + log2 l) * ln2.
#pragma unroll
  for (int c = 0; c < QC; ++c) {
    const float ls = group4_sum(lsum[c]);
    const int qi = wq0 + 16 * c + (l & 15);
    if (qi < T) {
      const float inv = 1.f / ls;
      bf16* orow = O + ((long long)b * T + qi) * ldo + (long long)h * HD;
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        bf16x4 v = {(bf16)(o[c][d][0] * inv), (bf16)(o[c][d][1] * inv), (bf16)(o[c][d][2] * inv),
                    (bf16)(o[c][d][3] * inv)};
        *reinterpret_cast<bf16x4*>(orow + 16 * d + 4 * g) = v;
      }
      if (g == 0) LSE[((long long)b * H + h) * T + qi] = (m[c] + __log2f(ls)) * kLn2;
    }
  }
}

// ============================================================ forward (32x32x16 MFMA) ==
// v_mfma_f32_32x32x16_bf16 holds the SIMD's vector issue for 8 of its 32 cycles, the
// 16x16x32 form for 8 of 16: per FLOP the 32x32 shape leaves 3x the issue slots for the
// softmax VALU that runs beside it (MI355X_MICROARCH.md, 'vector-instruction ISSUE cost'),
// which is what bounds attention at head_dim 64.  Block: 4 waves x 32 queries; K/V tiles of
// 64 keys by LDS-DMA into a 3-deep ring (tile t+2 in flight while t is computed).
//
//  * S^T = K Q^T per wave: 2 key halves x HD/16 k-steps; lane (r = l&31, h = l>>5) owns query
//    column r and keys 8(i>>2) + 4h + (i&3) of each half (C/D map), so registers 8s..8s+7 of
//    a half are, packed to bf16, directly the B operand of k-step s of O^T = V^T P^T (guide
//    §3 'An accumulator tile as the next MFMA's operand'); the permuted k order is absorbed
//    by the V^T fragment's transposed reads (rows 16s + 4h + 0..3 and + 8..11).
//  * K and V tiles carry separate XOR swizzles, each conflict-free for its one read pattern:
//    K rows by ds_read_b128 (16-lane groups span 16 rows), V by ds_read_b64_tr_b16 (32-lane
//    groups span 4 rows x 64 B).
//  * online softmax with the deferred rescale of attn_fwd_k (m moves only when a row's tile max
//    exceeds it by 2^8); the row statistics of lanes l and l^32 (same query, other keys) meet
//    in one v_permlane32_swap, only on that rare branch and in the epilogue.
template <int HD>
__device__ __forceinline__ int swz_k(int r, int ch) {
  return HD == 64 ? (ch ^ ((r >> 1) & 7)) : (ch ^ (r & 15));
}
template <int HD>
__device__ __forceinline__ int swz_v(int r, int ch) {
  return HD == 64 ? (ch ^ (((r >> 1) & 1) << 2)) : (ch ^ ((r & 3) << 2));
}

// Per-lane source offsets of a wave's K/V pieces (the swizzle is a function of the tile
// row, so they are tile-invariant); a tile's pieces then cost one scalar descriptor each.
template <int HD, int NW>
struct KvDma3 {
  static constexpr int CPR = HD / 8, TILE = 64 * HD * 2, P = 2 * TILE / 1024, PW = P / NW;
  static_assert(PW >= 2 && PW * NW == P, "pieces must divide over the waves");
  unsigned voff[PW];
  __device__ __forceinline__ void init(long long ldk, long long ldv) {
    const int l = lane_id(), wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const bool isv = i >= PW / 2;                 // pieces wave + NW i: K first, then V
      const int jj = wave + NW * i - (isv ? P / 2 : 0);
      const int pos = jj * 64 + l;
      const int r = pos / CPR, cp = pos % CPR;
      const int ch = isv ? swz_v<HD>(r, cp) : swz_k<HD>(r, cp);   // XOR swizzles are involutions
      voff[i] = (unsigned)(((long long)r * (isv ? ldv : ldk) + ch * 8) * 2);
    }
  }
  // tile rows [kv0, kv0 + 64) -> stage (K at 0, V at TILE); rows >= T fall outside the
  // descriptor's range and read as zeros.
  __device__ __forceinline__ void issue(const bf16* kbase, const bf16* vbase, long long ldk, long long ldv, int T,
                                        int kv0, char* stage) const {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned ks = (unsigned)(((long long)(T - 1 - kv0) * ldk + HD) * 2);
    const unsigned vs = (unsigned)(((long long)(T - 1 - kv0) * ldv + HD) * 2);
    const __amdgpu_buffer_rsrc_t rk =
        __builtin_amdgcn_make_buffer_rsrc((void*)(kbase + (long long)kv0 * ldk), (short)0, (int)ks, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv =
        __builtin_amdgcn_make_buffer_rsrc((void*)(vbase + (long long)kv0 * ldv), (short)0, (int)vs, 0x00020000);
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const bool isv = i >= PW / 2;
      const int jj = wave + NW * i - (isv ? P / 2 : 0);
      dma16(isv ? rv : rk, stage + (isv ? TILE : 0) + jj * 1024, voff[i]);
    }
  }
};

// DIAG = 1: per-wave s_memtime split (wait + barrier / QK^T + mask + max / exp + pack / P.V /
// block starts / block ends) into diag[block][wave][10] (timing build only; the stamps cost
// ~10 %).
__device__ __forceinline__ unsigned long long stamp_dep(float dep) {
  unsigned long long t;
  asm volatile("; stamp after %0" ::"v"(dep));
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
__device__ __forceinline__ unsigned long long realtime() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// Work cursor of the persistent forward: item it = (b, h, pair p) -> query blocks nqb-1-p
// (heavy) then p (light), equal causal work for every pair; item it serves (b, h) index
// 8 (it / 8 / NP) + it % 8, so with a grid that is a multiple of 8 all items of a head run on
// one XCD (workgroups are dealt to the XCDs round-robin) and its K / V stay in that L2.
struct FwdCur {
  int it, sub, t, nkv, qb, bh;
};
__device__ __forceinline__ bool fwd_cur_fix(FwdCur& c, int n_items, int NP, int nqb, int BH, int T, int causal) {
  while (c.it < n_items) {
    const int rest = c.it >> 3, p = rest % NP;
    c.bh = (rest / NP) * 8 + (c.it & 7);
    if (c.bh < BH) {
      const int nsub = (nqb - 1 - p == p) ? 1 : 2;
      if (c.sub < nsub) {
        c.qb = c.sub == 0 ? nqb - 1 - p : p;
        c.nkv = ((causal ? min(T, (c.qb + 1) * 128) : T) + 63) / 64;
        return true;
      }
    }
    c.it += gridDim.x;
    c.sub = 0;
    c.t = 0;
  }
  return false;
}
__device__ __forceinline__ bool fwd_cur_next(FwdCur& c, int n_items, int NP, int nqb, int BH, int T, int causal) {
  if (++c.t < c.nkv) return true;
  c.t = 0;
  ++c.sub;
  return fwd_cur_fix(c, n_items, NP, nqb, BH, T, causal);
}

// Persistent: each workgroup walks items (fwd_cur_fix) one query block at a time.  The K/V
// tiles of a block come by LDS-DMA into a 3-slot ring two tiles ahead; the ring numbering runs
// on across blocks, so in a block's last tile (after its QK^T, when Q is dead and the two
// slots ahead are free) the workgroup already fetches the next block's Q (buffer loads, rows
// >= T read as zeros) and its first two tiles, and the fetch flies under the softmax, P.V and
// epilogue.  O / LSE go out as buffer stores (rows >= T dropped by the descriptor), so every
// wave issues the same vector-memory operations and the counted vmcnt waits are exact.
// RSM: the row sum of P by one more MFMA per 16-key step (an all-ones A operand: O^T rows of
// ones), in place of the per-element adds beside the MFMAs (A/B: impl 6).
// MF: the softmax scale and the running max folded into the MFMAs (impl 8): Q is scaled by
// scale * log2(e) once per block in registers, and one more 32x32x16 MFMA per key half adds
// -m (a B column [-m, 0, ...] against an A column of ones) to the score accumulator, so
// p = exp2(s) needs no per-element fma; m is kept bf16-exact (it is only a shift).
template <int HD, int DIAG = 0, bool RSM = false, bool MF = false>
__global__ __launch_bounds__(256, (HD > 64 ? 1 : 2)) void attn_fwd3_k(const bf16* __restrict__ Q, const bf16* __restrict__ K,
                                                     const bf16* __restrict__ V, bf16* __restrict__ O,
                                                     float* __restrict__ LSE, int T, int H, int BH, long long ldq,
                                                     long long ldk, long long ldv, long long ldo, float scale,
                                                     int causal, unsigned long long* __restrict__ diag = nullptr) {
  constexpr int NW = 4, BQ = 32 * NW, BKV = 64, KS = HD / 16, DTN = HD / 32, RB = HD * 2;
  constexpr int TILE = BKV * RB, STAGE = 2 * TILE, NST = 3;
  constexpr int PW = 2 * TILE / 1024 / NW;   // DMA pieces per wave per tile
  constexpr int ST = DTN * 4 + 1;            // stores per wave per query block (O + LSE)
  static_assert(PW + ST < 64, "vmcnt range");
  __shared__ __attribute__((aligned(1024))) char smem[NST * STAGE];
  const int nqb = (T + BQ - 1) / BQ;
  const int NP = (nqb + 1) / 2;
  const int n_items = (BH + 7) / 8 * 8 * NP;
  const int wave = threadIdx.x >> 6, l = lane_id(), r32 = l & 31, hf = l >> 5, g16 = l >> 4, i16 = l & 15;
  const float c2 = scale * kLog2e;

  unsigned long long d_acc[6] = {0, 0, 0, 0, 0, 0}, d_t0 = 0, d_t1 = 0, d_start = 0, d_rt0 = 0, d_sb = 0;
  if constexpr (DIAG) {
    d_start = stamp_dep(0.f);
    d_rt0 = realtime();
  }

  FwdCur c = {(int)blockIdx.x, 0, 0, 0, 0, 0};
  if (!fwd_cur_fix(c, n_items, NP, nqb, BH, T, causal)) return;   // block-uniform
  KvDma3<HD, NW> dma;
  dma.init(ldk, ldv);
  int koff[2][KS];   // K A-fragment (half kh, k-step ks): row 32 kh + r32, chunk 2 ks + hf
#pragma unroll
  for (int kh = 0; kh < 2; ++kh)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int r = 32 * kh + r32;
      koff[kh][ks] = r * RB + (swz_k<HD>(r, 2 * ks + hf) << 4);
    }
  // V^T fragment reads: rows 16 k4 + 4 hf + (i16 >> 2) [+ 8], d columns 32 dt + 16 (g16 & 1) +
  // 4 (i16 & 3); swz_v depends on row bits the 16 k4 / + 8 steps never touch, so a lane has
  // one offset per dt and the row steps ride the read's offset field
  int voff[DTN];
#pragma unroll
  for (int dt = 0; dt < DTN; ++dt) {
    const int row = 4 * hf + (i16 >> 2);
    const int col = 32 * dt + 16 * (g16 & 1) + 4 * (i16 & 3);
    voff[dt] = row * RB + (swz_v<HD>(row, col >> 3) << 4) + (col & 7) * 2;
  }
  const unsigned qspan = (unsigned)(((long long)(T - 1) * ldq + HD) * 2);
  const unsigned ospan = (unsigned)(((long long)(T - 1) * ldo + HD) * 2);
  bf16x8 qf[KS];
  // next block's Q (Q^T operand: lane holds Q[q0 + 32 wave + r32][16 ks + 8 hf + j]) and its
  // first two tiles into ring slots s0, s0 + 1
  auto fetch_block = [&](const FwdCur& n, int s0) __attribute__((always_inline)) {
    const int b = n.bh / H, h = n.bh % H;
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Q + (long long)b * T * ldq + (long long)h * HD), (short)0, (int)qspan, 0x00020000);
    const int qi = n.qb * BQ + wave * 32 + r32;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const unsigned off = (unsigned)(((long long)qi * ldq + 16 * ks + 8 * hf) * 2);
      asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(qf[ks]) : "v"(off), "s"(rq));
    }
    const bf16* kb = K + (long long)b * T * ldk + (long long)h * HD;
    const bf16* vb = V + (long long)b * T * ldv + (long long)h * HD;
    dma.issue(kb, vb, ldk, ldv, T, 0, smem + s0 * STAGE);
    if (n.nkv > 1) dma.issue(kb, vb, ldk, ldv, T, BKV, smem + (s0 + 1 == NST ? 0 : s0 + 1) * STAGE);
  };

  fetch_block(c, 0);
  int base = 0;          // ring slot of the block's tile 0
  bool firstb = true;
  while (true) {
    const int b = c.bh / H, h = c.bh % H;
    const bf16* kb = K + (long long)b * T * ldk + (long long)h * HD;
    const bf16* vb = V + (long long)b * T * ldv + (long long)h * HD;
    const int nkv = c.nkv, q0 = c.qb * BQ, wq0 = q0 + wave * 32, qi = wq0 + r32;
    FwdCur n = c;
    n.t = nkv - 1;
    const bool nv = fwd_cur_next(n, n_items, NP, nqb, BH, T, causal);   // the next block, if any
    f32x16 o[DTN], osum;
#pragma unroll
    for (int d = 0; d < DTN; ++d)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[d][i] = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) osum[i] = 0.f;
    float m = MF ? 0.f : -INFINITY, lsum = 0.f;
    // MF: the extra k-step's operands (A: lanes 0-31 hold k = 0 of a key row = 1; B: lanes 0-31
    // hold k = 0 of a query column = -m)
    bf16x8 kx = {}, qx = {};
    if constexpr (MF) {
      if (hf == 0) kx[0] = (bf16)1.f;
    }
    int slot = base;
    for (int t = 0; t < nkv; ++t) {
      // tile t landed; what was issued after its DMA may still fly: the next tile (PW) and,
      // for tiles 0 / 1 of all but the first block, the previous block's stores (ST)
      if constexpr (DIAG) d_t0 = stamp_dep(0.f);
      const bool nxt = t + 1 < nkv;
      if (t >= 2 || firstb) {
        if (nxt) wait_vmcnt<PW>();
        else wait_vmcnt<0>();
      } else {
        if (nxt) wait_vmcnt<PW + ST>();
        else wait_vmcnt<ST>();
      }
      __builtin_amdgcn_s_barrier();
      if constexpr (DIAG) {
        d_t1 = stamp_dep(0.f);
        d_acc[0] += d_t1 - d_t0;
      }
      const char* lk = smem + slot * STAGE;
      const char* lv = lk + TILE;
      const int s1 = slot + 1 == NST ? 0 : slot + 1, s2 = s1 + 1 == NST ? 0 : s1 + 1;
      if (t + 2 < nkv) dma.issue(kb, vb, ldk, ldv, T, (t + 2) * BKV, smem + s2 * STAGE);
      if constexpr (MF) {
        if (t == 0) {
          // this block's Q landed (the wait above): Q' = bf16(Q scale log2 e).  (The empty asm
          // orders the reads of the asm-loaded registers after the wait.)
          asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]));
          if constexpr (KS > 4) asm volatile("" : "+v"(qf[KS - 4]), "+v"(qf[KS - 3]), "+v"(qf[KS - 2]), "+v"(qf[KS - 1]));
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int j = 0; j < 8; ++j) qf[ks][j] = (bf16)((float)qf[ks][j] * c2);
        }
      }
      const int kv0 = t * BKV;
      const bool last = t + 1 == nkv;
      const bool active = !causal || kv0 <= wq0 + 31;   // wave-uniform
      f32x16 s[2];
      if (active) {
        if constexpr (HD > 64) {
          // one wave per SIMD (hd 128): key half 0's K fragments all read before its first
          // MFMA, half 1's under half 0's MFMAs (at hd 64, three waves per SIMD leave no
          // register room for it and the other waves hide the LDS latency)
          bf16x8 ka[KS], kb[KS];
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) ka[ks] = *reinterpret_cast<const bf16x8*>(lk + koff[0][ks]);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < 16; ++i) s[0][i] = 0.f;
          if constexpr (MF) s[0] = MFMA32(kx, qx, s[0]);
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            s[0] = MFMA32(ka[ks], qf[ks], s[0]);
            kb[ks] = *reinterpret_cast<const bf16x8*>(lk + koff[1][ks]);
            __builtin_amdgcn_sched_barrier(0);
          }
#pragma unroll
          for (int i = 0; i < 16; ++i) s[1][i] = 0.f;
          if constexpr (MF) s[1] = MFMA32(kx, qx, s[1]);
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) s[1] = MFMA32(kb[ks], qf[ks], s[1]);
        } else {
#pragma unroll
          for (int kh = 0; kh < 2; ++kh) {
#pragma unroll
            for (int i = 0; i < 16; ++i) s[kh][i] = 0.f;
            if constexpr (MF) s[kh] = MFMA32(kx, qx, s[kh]);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
              const bf16x8 kf = *reinterpret_cast<const bf16x8*>(lk + koff[kh][ks]);
              s[kh] = MFMA32(kf, qf[ks], s[kh]);
            }
          }
        }
      }
      if (last && nv) {
        __builtin_amdgcn_sched_barrier(0);
        fetch_block(n, s1);   // Q is dead; slots s1, s2 held tiles t-2, t-1 (all waves past them)
      }
      if (active) {
        // V^T fragments (asm transposed reads: no compiler vmcnt(0) with the DMA in flight)
        __builtin_amdgcn_sched_barrier(0);
        constexpr int NVH = 2 * DTN * 4;
        s16x4 vh[(NVH + 15) / 16 * 16];
#pragma unroll
        for (int dt = 0; dt < DTN; ++dt) {
          const char* vb = lv + voff[dt];
#pragma unroll
          for (int k4 = 0; k4 < 4; ++k4) {
            vh[2 * (dt * 4 + k4)] = ds_tr16_off(vb, 16 * k4 * RB);
            vh[2 * (dt * 4 + k4) + 1] = ds_tr16_off(vb, (16 * k4 + 8) * RB);
          }
        }
        const bool need_mask = __builtin_amdgcn_readfirstlane(
            (int)((causal && kv0 + BKV - 1 > wq0) || (kv0 + BKV > T)));
        if (need_mask) {
          // key kv0 + 32 kh + 8 (i>>2) + 4 hf + (i&3) is valid iff its tile offset <= lim
          const int lim = (causal ? min(qi, T - 1) : T - 1) - kv0 - 4 * hf;
#pragma unroll
          for (int kh = 0; kh < 2; ++kh)
#pragma unroll
            for (int i = 0; i < 16; ++i)
              s[kh][i] = (32 * kh + 8 * (i >> 2) + (i & 3) > lim) ? -INFINITY : s[kh][i];
        }
        // lane max as a 4-way tree of v_max3 (short dependency chains; asm: hipcc otherwise puts a
        // canonicalising v_max in front of fmaxf on MFMA results)
        float mq[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int h = j >> 1, o = 8 * (j & 1);
          mq[j] = vmax3(vmax3(vmax3(s[h][o], s[h][o + 1], s[h][o + 2]), s[h][o + 3], s[h][o + 4]), s[h][o + 5],
                        s[h][o + 6]);
          mq[j] = vmax2(mq[j], s[h][o + 7]);
        }
        const float mx = vmax2(vmax3(mq[0], mq[1], mq[2]), mq[3]);
        if constexpr (DIAG) {
          const unsigned long long t2 = stamp_dep(mx);
          d_acc[1] += t2 - d_t1;
          d_t1 = t2;
        }
        // deferred rescale (as attn_fwd_k): m moves only when a row's tile max exceeds it by 2^8;
        // every visited tile has a valid key for every query row (kv0 <= wq0), so m is finite
        // after the first tile
        constexpr float kDefer = 8.f;
        if constexpr (MF) {
          // s = S' - m already; the first tile sets m (the plain form's -inf start), later ones
          // move it only past the defer threshold.  m stays bf16-exact (the B column's -m).
          if (t == 0 || __builtin_amdgcn_ballot_w64(mx > kDefer) != 0) {
            const float mr = pair_max(mx);
            const float mnew = (t == 0 || mr > kDefer) ? (float)(bf16)(m + mr) : m;
            const float d = mnew - m;
            if (t > 0) {
              const float alpha = __builtin_amdgcn_exp2f(-d);
              lsum *= alpha;
#pragma unroll
              for (int dd = 0; dd < DTN; ++dd) o[dd] *= alpha;
            }
#pragma unroll
            for (int kh = 0; kh < 2; ++kh) s[kh] -= d;
            m = mnew;
            if (hf == 0) qx[0] = (bf16)(-m);
          }
        } else if (__builtin_amdgcn_ballot_w64(mx * c2 > m + kDefer) != 0) {
          const float mr = pair_max(mx) * c2;   // both lanes of a row decide together
          const float mnew = mr > m + kDefer ? mr : m;
          const float alpha = mnew == m ? 1.f : __builtin_amdgcn_exp2f(m - mnew);
          m = mnew;
          lsum *= alpha;
          if constexpr (RSM) osum *= alpha;
#pragma unroll
          for (int d = 0; d < DTN; ++d) o[d] *= alpha;
        }
        // row sum in 4 scalar chains (single v_add_f32: no packed adds beside the MFMAs)
        float ps[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int i = 0; i < 16; i += 2) {
            const float e0 = __builtin_amdgcn_exp2f(MF ? s[kh][i] : fmaf(s[kh][i], c2, -m));
            const float e1 = __builtin_amdgcn_exp2f(MF ? s[kh][i + 1] : fmaf(s[kh][i + 1], c2, -m));
            s[kh][i] = e0;
            s[kh][i + 1] = e1;
            if constexpr (!RSM) {
              ps[(i >> 1) & 3] = vaddf(ps[(i >> 1) & 3], e0);
              ps[((i >> 1) + 2) & 3] = vaddf(ps[((i >> 1) + 2) & 3], e1);
            }
          }
        if constexpr (!RSM) lsum += (ps[0] + ps[1]) + (ps[2] + ps[3]);
        bf16x8 pk[4];
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4)
#pragma unroll
          for (int j = 0; j < 8; ++j) pk[k4][j] = (bf16)s[k4 >> 1][8 * (k4 & 1) + j];
        if constexpr (DIAG) {
          const unsigned long long t3 = stamp_dep(__builtin_bit_cast(float, __builtin_bit_cast(u32x4, pk[3])[0]));
          d_acc[2] += t3 - d_t1;
          d_t1 = t3;
        }
#pragma unroll
        for (int w = 0; w < (NVH + 15) / 16; ++w) tr_wait8(*reinterpret_cast<s16x4(*)[16]>(&vh[16 * w]));
#pragma unroll
        for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
          for (int k4 = 0; k4 < 4; ++k4) {
            const bf16x8 vf = tr_join(vh[2 * (dt * 4 + k4)], vh[2 * (dt * 4 + k4) + 1]);
            o[dt] = MFMA32(vf, pk[k4], o[dt]);
          }
        if constexpr (RSM) {
          bf16x8 ones;
#pragma unroll
          for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.f;
#pragma unroll
          for (int k4 = 0; k4 < 4; ++k4) osum = MFMA32(ones, pk[k4], osum);
        }
        if constexpr (DIAG) d_acc[3] += stamp_dep(o[DTN - 1][15]) - d_t1;
      }
      slot = s1;
    }
    // epilogue: O[q][d] = O^T[d][q] / l (lane: rows 32 dt + 8 g + 4 hf + 0..3 of column q);
    // lse = (m + log2 l) ln 2.  Buffer stores: rows >= T fall outside the descriptor.
    if constexpr (DIAG) d_sb = stamp_dep(0.f);
    {
      const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(O + (long long)b * T * ldo + (long long)h * HD), (short)0, (int)ospan, 0x00020000);
      const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(LSE + (long long)c.bh * T), (short)0, T * 4, 0x00020000);
      const float ls = RSM ? osum[0] : pair_sum(lsum);   // (every osum row is the row sum)
      const float inv = 1.f / ls;
#pragma unroll
      for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          bf16x4 v = {(bf16)(o[dt][4 * g] * inv), (bf16)(o[dt][4 * g + 1] * inv), (bf16)(o[dt][4 * g + 2] * inv),
                      (bf16)(o[dt][4 * g + 3] * inv)};
          const unsigned off = (unsigned)(((long long)qi * ldo + 32 * dt + 8 * g + 4 * hf) * 2);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), ro, off, 0, 0);
        }
      if (hf == 0)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((m + __log2f(ls)) * kLn2), rl, (unsigned)qi * 4u, 0, 0);
    }
    if constexpr (DIAG) d_acc[5] += stamp_dep(0.f) - d_sb;
    if (!nv) break;
    base = slot;           // the slot after the last tile's
    c = n;
    firstb = false;
  }
  if constexpr (DIAG) {
    if (l == 0) {
      unsigned long long* dp = diag + ((long long)blockIdx.x * 4 + wave) * 10;
      dp[0] = d_acc[0];
      dp[1] = d_acc[1];
      dp[2] = d_acc[2];
      dp[3] = d_acc[3];
      dp[4] = d_start;
      dp[5] = stamp_dep(0.f);
      dp[6] = d_rt0;
      dp[7] = realtime();
      dp[8] = d_acc[4];
      dp[9] = d_acc[5];
    }
  }
}

// Optional inverse RoPE fused into the dQ / dK stores: tab[pos][HD] = [cos | sin] of the
// HD/2 frequencies; column d < HD/2 pairs with d + HD/2, which lives in the same lane
// (accumulator tile d + DT/2), so the transpose rotation is applied in registers.
//   dx1 = dy1 c + dy2 s ;  dx2 = dy2 c - dy1 s
// ================================================================ bwd: dK, dV (LDS-DMA) ==
// Same math and block shape as attn_bwd_dkdv_k (4 waves x 16 keys, query tiles of 64), but
// Q / dO tiles and their LSE / delta rows arrive by LDS-DMA into a 3-deep ring: tile t+2
// is in flight while tile t is computed (the register-staged kernel waited ~45 % of its
// wave cycles on the one-tile-ahead loads, profiles/r1_v5_attn_bwd_pmc.txt).  Every wave
// issues the same 5 DMA instructions per tile (4 x 1 KiB pieces of Q/dO, one 256-B row of
// LSE or delta or an out-of-range dummy), so one counted vmcnt serves all waves.
template <int HD>
__device__ __forceinline__ void qdo_dma(__amdgpu_buffer_rsrc_t rq, __amdgpu_buffer_rsrc_t rdo,
                                        __amdgpu_buffer_rsrc_t rl, __amdgpu_buffer_rsrc_t rd, char* stage, int q0,
                                        int T, long long ldq, long long lddo) {
  constexpr int CPR = HD / 8;
  constexpr int TILE = 64 * HD * 2;
  constexpr int P = 2 * TILE / 1024;          // 1 KiB pieces per Q + dO tile
  constexpr int PW = P / 4;                   // per wave (4 waves)
  const int l = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int j = wave + 4 * i;
    const bool isdo = j >= P / 2;
    const int jj = isdo ? j - P / 2 : j;
    const int pos = jj * 64 + l;
    const int r = pos / CPR, cp = pos % CPR;
    const int ch = ((sw_off<HD>(r, cp) - r * HD * 2) >> 4);
    const int row = q0 + r;
    const long long ld = isdo ? lddo : ldq;
    const unsigned off = row < T ? (unsigned)(((long long)row * ld + ch * 8) * 2) : kOOB;
    dma16(isdo ? rdo : rq, stage + (isdo ? TILE : 0) + jj * 1024, off);
  }
  // stats: wave 0 -> LSE[q0..q0+63], wave 1 -> delta, waves 2/3 -> dummy (OOB) into a pad slot
  char* st = stage + 2 * TILE;
  const unsigned soff = (wave < 2 && q0 + l < T) ? (unsigned)((q0 + l) * 4) : kOOB;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(wave == 1 ? rd : rl,
                                           (__attribute__((address_space(3))) void*)(st + (wave < 2 ? wave : 2) * 256),
                                           4, soff, 0, 0, 0);
}

// qdo_dma with the per-lane part of every DMA offset computed once per kernel: per tile only
// the wave-uniform q0 * ld term and the tail-row test remain (the generic form re-derived
// the swizzled chunk / row split of every piece for every tile: ~50 VALU + ~60 SALU a tile).
template <int HD>
struct QdoPlan {
  static constexpr int TILE = 64 * HD * 2;
  static constexpr int PW = 2 * TILE / 1024 / 4;   // 1 KiB pieces per wave
  unsigned base[PW];                               // (r * ld + ch * 8) * 2
  int r[PW];                                       // row within the tile
  __device__ void init(long long ldq, long long lddo) {
    constexpr int CPR = HD / 8;
    constexpr int P = 2 * TILE / 1024;
    const int l = lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int j = wave + 4 * i;
      const bool isdo = i >= P / 8;             // (waves < 4: piece j < P/2 <=> i < P/8)
      const int jj = isdo ? j - P / 2 : j;
      const int pos = jj * 64 + l;
      const int rr = pos / CPR, cp = pos % CPR;
      const int ch = ((sw_off<HD>(rr, cp) - rr * HD * 2) >> 4);
      r[i] = rr;
      base[i] = (unsigned)(((long long)rr * (isdo ? lddo : ldq) + ch * 8) * 2);
    }
  }
  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rq, __amdgpu_buffer_rsrc_t rdo,
                                        __amdgpu_buffer_rsrc_t rl, __amdgpu_buffer_rsrc_t rd, char* stage, int q0,
                                        int T, long long ldq, long long lddo) const {
    constexpr int P = 2 * TILE / 1024;
    const int l = lane_id();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const unsigned qoff = (unsigned)((long long)q0 * ldq * 2), dooff = (unsigned)((long long)q0 * lddo * 2);
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int j = wave + 4 * i;
      const bool isdo = i >= P / 8;             // compile-time per unrolled i
      const int jj = isdo ? j - P / 2 : j;
      const unsigned off = q0 + r[i] < T ? base[i] + (isdo ? dooff : qoff) : kOOB;
      dma16(isdo ? rdo : rq, stage + (isdo ? TILE : 0) + jj * 1024, off);
    }
    char* st = stage + 2 * TILE;
    const unsigned soff = (wave < 2 && q0 + l < T) ? (unsigned)((q0 + l) * 4) : kOOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(wave == 1 ? rd : rl,
                                             (__attribute__((address_space(3))) void*)(st + (wave < 2 ? wave : 2) * 256),
                                             4, soff, 0, 0, 0);
  }
};

template <int HD>
__global__ __launch_bounds__(256, (HD > 64 ? 1 : 2)) void attn_bwd_dkdv2_k(
    const bf16* __restrict__ Q, const bf16* __restrict__ K, const bf16* __restrict__ V, const bf16* __restrict__ dO,
    const float* __restrict__ LSE, const float* __restrict__ DELTA, bf16* __restrict__ dK, bf16* __restrict__ dV,
    int T, int H, long long ldq, long long ldk, long long ldv, long long lddo, long long lddk, long long lddv,
    float scale, int causal, const int64_t* __restrict__ rpos, const float* __restrict__ rtab,
    float* __restrict__ BPK, float* __restrict__ BPV) {
  // LSE here = -lse/scale and DELTA = -delta per query row (written by attn_bwd_dq_k).
  // BPK / BPV (optional): each wave's column sums of its stored dK / dV rows, row
  // ((h * B + b) * nkb + kb) * 4 + wave of a [H * B * nkb * 4, HD] partial (k / v bias grad).
  constexpr int BKV = 64, BQ = 64, KT = HD / 32, DT = HD / 16;
  constexpr int TILE = BQ * HD * 2;
  constexpr int BUF = 2 * TILE + 1024;        // Q, dO, lse, delta, dummy slot (1 KiB aligned stages)
  constexpr int NST = 3;
  constexpr int PWV = 2 * TILE / 1024 / 4 + 1;  // DMA instructions per wave per tile
  __shared__ __attribute__((aligned(1024))) char smem[NST * BUF];
  // XCD-aware order: the key blocks of one (b, h) -- which all stream its Q / dO -- run on one
  // XCD (one L2).
  const int xl = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
  const int kb = xl % gridDim.x;
  const int bh = xl / gridDim.x, b = bh / H, h = bh % H;
  const int k0 = kb * BKV;
  const int wave = threadIdx.x >> 6, l = lane_id(), g = l >> 4;
  const int wk0 = k0 + wave * 16;
  const float c2 = scale * kLog2e;

  const bf16* qbase = Q + (long long)b * T * ldq + (long long)h * HD;
  const bf16* dobase = dO + (long long)b * T * lddo + (long long)h * HD;
  const float* lse_b = LSE + ((long long)b * H + h) * T;
  const float* del_b = DELTA + ((long long)b * H + h) * T;
  const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
      (void*)qbase, (short)0, (int)(((long long)(T - 1) * ldq + HD) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rdo = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dobase, (short)0, (int)(((long long)(T - 1) * lddo + HD) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc((void*)lse_b, (short)0, T * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)del_b, (short)0, T * 4, 0x00020000);

  const int qstart = causal ? (k0 / BQ) * BQ : 0;
  const int nq = (T - qstart + BQ - 1) / BQ;
  QdoPlan<HD> plan;
  plan.init(ldq, lddo);
  if (nq > 0) plan.issue(rq, rdo, rl, rd, smem, qstart, T, ldq, lddo);
  if (nq > 1) plan.issue(rq, rdo, rl, rd, smem + BUF, qstart + BQ, T, ldq, lddo);

  bf16x8 kf[KT], vf[KT];
  {
    const int ki = wk0 + (l & 15);
#pragma unroll
    for (int kk = 0; kk < KT; ++kk) {
      bf16x8 a = {}, c = {};
      if (ki < T) {
        a = *reinterpret_cast<const bf16x8*>(K + ((long long)b * T + ki) * ldk + (long long)h * HD + 32 * kk + 8 * g);
        c = *reinterpret_cast<const bf16x8*>(V + ((long long)b * T + ki) * ldv + (long long)h * HD + 32 * kk + 8 * g);
      }
      kf[kk] = a;
      vf[kk] = c;
    }
  }
  f32x4 dk[DT], dv[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) {
    dk[d] = (f32x4){0.f, 0.f, 0.f, 0.f};
    dv[d] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }

  int cur = 0;
  for (int t = 0; t < nq; ++t) {
    if (t + 1 < nq) wait_vmcnt<PWV>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    const char* lq = smem + cur * BUF;
    const char* ldo_ = lq + TILE;
    const float* ls = reinterpret_cast<const float*>(lq + 2 * TILE);
    const float* ds = ls + BQ;
    int nb = cur + 2;
    if (nb >= NST) nb -= NST;
    cur = (cur + 1 == NST) ? 0 : cur + 1;
    const int qq0 = qstart + t * BQ;
    if (t + 2 < nq) plan.issue(rq, rdo, rl, rd, smem + nb * BUF, qq0 + 2 * BQ, T, ldq, lddo);
    const bool wave_active = !causal || (qq0 + BQ - 1 >= wk0);
    if (!wave_active) continue;
    // Row constants as the initial accumulators (rows = queries 16qt + 4g + j): S' = QK^T -
    // lse/scale and dP' = dO V^T - delta, so p = exp2(c2 S') and dS = p dP' need no per-element
    // subtraction (the dQ kernel wrote -lse/scale and -delta).
    f32x4 s[4], dp[4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      s[qt] = *reinterpret_cast<const f32x4*>(ls + 16 * qt + 4 * g);
      dp[qt] = *reinterpret_cast<const f32x4*>(ds + 16 * qt + 4 * g);
#pragma unroll
      for (int kk = 0; kk < KT; ++kk) {
        s[qt] = MFMA(row_frag<HD>(lq, 16 * qt, 32 * kk), kf[kk], s[qt]);
        dp[qt] = MFMA(row_frag<HD>(ldo_, 16 * qt, 32 * kk), vf[kk], dp[qt]);
      }
    }
    // transposed dO fragments for dV (asm reads: see tr_frag_asm) land during the softmax; the
    // Q fragments for dK are read after the dV MFMAs are issued (two batches of 2*DT halves
    // keep the kernel at 3 waves/SIMD instead of holding both across the softmax).
    __builtin_amdgcn_sched_barrier(0);
    constexpr int NH = 2 * DT * 2;             // 2 k-slots x DT fragments x 2 halves
    constexpr int NHP = (NH + 15) / 16 * 16;
    s16x4 th[NHP];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int d = 0; d < DT; ++d) tr_frag_asm<HD>(ldo_, 32 * ks, 16 * d, th[2 * (ks * DT + d)], th[2 * (ks * DT + d) + 1]);
    const int ki = wk0 + (l & 15);
    // The mask test is wave-uniform (readfirstlane) and only diagonal / tail tiles run the
    // per-element selects: branch-free v_cndmask there, nothing on the other tiles.
    const bool need_mask = __builtin_amdgcn_readfirstlane(
        (int)((causal && wk0 + 15 > qq0) || (qq0 + BQ > T) || (wk0 + 16 > T)));
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int j = 0; j < 4; ++j) s[qt][j] = __builtin_amdgcn_exp2f(s[qt][j] * c2);
    if (need_mask) {
#pragma unroll
      for (int qt = 0; qt < 4; ++qt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int qi = qq0 + 16 * qt + 4 * g + j;
          const bool z = (qi >= T) | (ki >= T) | (causal & (ki > qi));
          s[qt][j] = z ? 0.f : s[qt][j];
        }
    }
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int j = 0; j < 4; ++j) dp[qt][j] *= s[qt][j];
    bf16x8 pa[2], da[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      pa[ks] = pack_pt(s[2 * ks], s[2 * ks + 1]);
      da[ks] = pack_pt(dp[2 * ks], dp[2 * ks + 1]);
    }
#pragma unroll
    for (int w = 0; w < NHP / 16; ++w) tr_wait8(*reinterpret_cast<s16x4(*)[16]>(&th[16 * w]));
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int d = 0; d < DT; ++d) dv[d] = MFMA(pa[ks], tr_join(th[2 * (ks * DT + d)], th[2 * (ks * DT + d) + 1]), dv[d]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int d = 0; d < DT; ++d) tr_frag_asm<HD>(lq, 32 * ks, 16 * d, th[2 * (ks * DT + d)], th[2 * (ks * DT + d) + 1]);
#pragma unroll
    for (int w = 0; w < NHP / 16; ++w) tr_wait8(*reinterpret_cast<s16x4(*)[16]>(&th[16 * w]));
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int d = 0; d < DT; ++d) dk[d] = MFMA(da[ks], tr_join(th[2 * (ks * DT + d)], th[2 * (ks * DT + d) + 1]), dk[d]);
  }
  wait_vmcnt<0>();
  // Write dK (scaled, inverse RoPE), dV: C layout col = d (l&15), rows = keys 4g + j.
#pragma unroll
  for (int d = 0; d < DT; ++d)
#pragma unroll
    for (int j = 0; j < 4; ++j) dk[d][j] *= scale;
  if (rpos) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ki = wk0 + 4 * g + j;
      if (ki < T) {
        KASSERT(rpos[(long long)b * T + ki] >= 0, "rope position at key %d", ki);
        const float* tr = rtab + rpos[(long long)b * T + ki] * HD;
#pragma unroll
        for (int d = 0; d < DT / 2; ++d) {
          const float c = tr[16 * d + (l & 15)], sn = tr[HD / 2 + 16 * d + (l & 15)];
          const float x1 = dk[d][j], x2 = dk[d + DT / 2][j];
          dk[d][j] = x1 * c + x2 * sn;
          dk[d + DT / 2][j] = x2 * c - x1 * sn;
        }
      }
    }
  }
#pragma unroll
  for (int d = 0; d < DT; ++d) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ki = wk0 + 4 * g + j;
      if (ki < T) {
        const long long col = (long long)h * HD + 16 * d + (l & 15);
        dK[((long long)b * T + ki) * lddk + col] = (bf16)dk[d][j];
        dV[((long long)b * T + ki) * lddv + col] = (bf16)dv[d][j];
      }
    }
  }
  if (BPK) {
    // Column sums over the wave's 16 keys (4 in-lane, then the 4 lane groups).
    float sk[DT], sv[DT];
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      sk[d] = 0.f;
      sv[d] = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (wk0 + 4 * g + j < T) {
          sk[d] += dk[d][j];
          sv[d] += dv[d][j];
        }
      }
      sk[d] += __shfl_xor(sk[d], 16, 64);
      sv[d] += __shfl_xor(sv[d], 16, 64);
      sk[d] += __shfl_xor(sk[d], 32, 64);
      sv[d] += __shfl_xor(sv[d], 32, 64);
    }
    // One partial row per wave (no block barrier: a wave that finishes early leaves).
    if (l < 16) {
      const long long row = (((long long)h * (gridDim.y / H) + b) * gridDim.x + kb) * 4 + wave;
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        BPK[row * HD + 16 * d + l] = sk[d];
        BPV[row * HD + 16 * d + l] = sv[d];
      }
    }
  }
}

// ======================================================== bwd: dK, dV (32x32x16 MFMA) ==
// Key on the lane (guide §B 'Attention backward'): a wave owns 32 keys; S = Q K^T and dP =
// dO V^T are computed with the queries as the 32x32 C rows, so their accumulators, packed to
// bf16, are directly the B operands of dV^T += dO^T P and dK^T += Q^T dS (registers 8s..8s+7
// = k-step s over queries, §3 'An accumulator tile as the next MFMA's operand'), and dK^T /
// dV^T stay in registers for the whole query sweep.  The row constants -lse/scale and
// -delta enter as the initial accumulators of S and dP (read from the LDS stage), so
// p = exp2(c2 S') and dS = p dP' need no per-element subtraction.  Q and dO tiles (64 rows)
// stream through a 3-slot LDS-DMA ring; each tile is read by rows (A operands of S / dP) and
// transposed (A operands of dV^T / dK^T, ds_read_b64_tr_b16), so both use one XOR swizzle
// that is conflict-free for both patterns (swz_u).  A workgroup = 4 waves x 32 keys and
// handles a causal pair of key blocks (p, nkb-1-p): the same work for every workgroup.
// DIAG = 1: per-wave s_memtime split into diag[block][wave][10]: wait + barrier / S, dP + first
// exp half / second exp half + mask + dS + packs / dO^T reads + dV^T / Q^T reads + dK^T /
// epilogues / prologues (K, V to registers) / tiles computed / start / end (timing build only:
// each stamp waits for the value it depends on).
// KSC: K scaled by scale log2(e) once per key block in registers and LSN = -lse log2(e) (the
// dQ kernel's KSC convention), so p = exp2(S') with no per-element multiply (impl 9, A/B:
// -1.5 % per call, nothing measurable per step, K rounded once more; impl 4 = the unscaled form).
template <int HD, int DIAG = 0, bool KSC = false>
__global__ __launch_bounds__(256, (HD > 64 ? 1 : 2)) void attn_bwd_dkdv3_k(
    const bf16* __restrict__ Q, const bf16* __restrict__ K, const bf16* __restrict__ V, const bf16* __restrict__ dO,
    const float* __restrict__ LSN, const float* __restrict__ NDEL, bf16* __restrict__ dK, bf16* __restrict__ dV,
    int T, int H, int BH, long long ldq, long long ldk, long long ldv, long long lddo, long long lddk,
    long long lddv, float scale, int causal, const int64_t* __restrict__ rpos, const float* __restrict__ rtab,
    float* __restrict__ BPK, float* __restrict__ BPV, unsigned long long* __restrict__ diag = nullptr,
    int prefetch = 1) {
  // LSN = -lse / scale and NDEL = -delta per query row (written by attn_bwd_dq3_k).  BPK / BPV
  // (optional): per (b, h, key block, wave) column sums of the stored dK / dV rows.
  static_assert(HD == 64 || HD == 128, "dK/dV v3: head_dim 64 or 128");
  constexpr int BK = 128, BQ = 64, KS = HD / 16, DTN = HD / 32, RB = HD * 2;
  constexpr int TILE = BQ * RB, BUF = 2 * TILE + 1024, NST = 3;
  constexpr int PWV = QdoDma3<HD>::PW + 1;   // DMA instructions per wave per tile
  // the ring, then each wave's epilogue rows (one array: a second LDS object made the compiler
  // wait for every LDS-DMA in flight before the ring reads)
  __shared__ __attribute__((aligned(1024))) char smem[NST * BUF + 4 * RowStage<HD>::BYTES];
  const int nkb = (T + BK - 1) / BK;
  const int NP = (nkb + 1) / 2;
  const int it = blockIdx.x;
  const int bh = (it >> 3) / NP * 8 + (it & 7), p = (it >> 3) % NP;
  if (bh >= BH) return;
  const int b = bh / H, h = bh % H;
  const int wave = threadIdx.x >> 6, l = lane_id(), r32 = l & 31, hf = l >> 5, g16 = l >> 4, i16 = l & 15;
  char* ep = smem + NST * BUF + wave * RowStage<HD>::BYTES;
  const float c2 = scale * kLog2e;
  const bf16* qbase = Q + (long long)b * T * ldq + (long long)h * HD;
  const bf16* dobase = dO + (long long)b * T * lddo + (long long)h * HD;
  const float* lsb = LSN + (long long)bh * T;
  const float* dlb = NDEL + (long long)bh * T;
  QdoDma3<HD> dma;
  dma.init(ldq, lddo);
  // lane-constant LDS offsets: row reads (row 32 qt + r32, chunk 2 ks + hf; the swizzle of
  // row + 32 equals that of row, so qt is an immediate) and transposed reads (rows 16 s4 + 4 hf
  // + (i16 >> 2) [+ 8], d columns 32 dt + 16 (g16 & 1) + 4 (i16 & 3); s4 is an immediate)
  int roff[KS], toff[DTN][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) roff[ks] = r32 * RB + (swz_u<HD>(r32, 2 * ks + hf) << 4);
#pragma unroll
  for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int row = 4 * hf + (i16 >> 2) + 8 * e;
      const int col = 32 * dt + 16 * (g16 & 1) + 4 * (i16 & 3);
      toff[dt][e] = row * RB + (swz_u<HD>(row, col >> 3) << 4) + (col & 7) * 2;
    }

  unsigned long long d_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, d_t0 = 0, d_start = 0;
  if constexpr (DIAG) d_start = stamp_dep(0.f);
  // The ring position runs on across the two key blocks: during the first block's last two
  // query tiles the second block's first two Q / dO tiles are fetched into the slots the
  // first block no longer needs, and its K / V rows into the K / V registers once the last
  // tile's S / dP MFMAs have consumed them -- the second block starts with its operands in
  // flight or landed instead of a cold prologue.
  const int kb1 = nkb - 1 - p;                       // the second key block (== p: none)
  const int qstart1 = causal ? ((kb1 * BK) / BQ) * BQ : 0;
  const int nq1 = (T - qstart1 + BQ - 1) / BQ;
  const int key1 = kb1 * BK + 32 * wave + r32;
  const int nq0 = (T - (causal ? ((p * BK) / BQ) * BQ : 0) + BQ - 1) / BQ;
  // (head_dim 64 only: at 128 the one-wave-per-SIMD kernel has no register to spare for it)
  const bool pre = HD == 64 && (prefetch & 1) && kb1 != p && nq1 > 0 && nq0 >= 2;  // (uniform)
  // A/B hook (prefetch >> 4 = n): odd workgroups start n x 8k cycles late, so the two workgroups
  // sharing a CU's SIMDs run their MFMA-heavy and VALU-heavy phases offset
  for (int sn = 0; sn < (blockIdx.x & 1) * (prefetch >> 4); ++sn) __builtin_amdgcn_s_sleep(127);
  bf16x8 kf[KS], vf[KS];
  auto load_kv = [&](int kk_) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 a_ = {}, c_ = {};
      if (kk_ < T) {
        a_ = *reinterpret_cast<const bf16x8*>(K + ((long long)b * T + kk_) * ldk + (long long)h * HD + 16 * ks + 8 * hf);
        c_ = *reinterpret_cast<const bf16x8*>(V + ((long long)b * T + kk_) * ldv + (long long)h * HD + 16 * ks + 8 * hf);
      }
      kf[ks] = a_;
      vf[ks] = c_;
    }
  };
  int cur = 0;
  for (int sub = 0; sub < 2; ++sub) {
    const int kb = sub == 0 ? p : nkb - 1 - p;
    if (sub == 1 && kb == p) break;
    if constexpr (DIAG) d_t0 = stamp_dep(0.f);
    if (sub == 1) __syncthreads();   // the previous key block's ring slots are read
    const int k0 = kb * BK, kw0 = k0 + 32 * wave, key = kw0 + r32;
    const int qstart = causal ? (k0 / BQ) * BQ : 0;
    const int nq = (T - qstart + BQ - 1) / BQ;
    const bool fetched = sub == 1 && pre;   // tiles 0 / 1 and K / V already on their way
    if (!fetched) {
      const int c1 = cur + 1 == NST ? 0 : cur + 1;
      if (nq > 0) dma.issue(qbase, dobase, lsb, dlb, ldq, lddo, T, qstart, smem + cur * BUF);
      if (nq > 1) dma.issue(qbase, dobase, lsb, dlb, ldq, lddo, T, qstart + BQ, smem + c1 * BUF);
      // K^T / V^T operands (B of S = Q K^T, dP = dO V^T): lane holds K[key][16 ks + 8 hf + j]
      load_kv(key);
    }
    wait_vmcnt<0>();
    if constexpr (KSC) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) kf[ks][j] = (bf16)((float)kf[ks][j] * c2);
    }
    if constexpr (DIAG) d_acc[6] += stamp_dep(__builtin_bit_cast(float, __builtin_bit_cast(u32x4, vf[KS - 1])[3])) - d_t0;
    f32x16 dkt[DTN], dvt[DTN];
#pragma unroll
    for (int d = 0; d < DTN; ++d)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        dkt[d][i] = 0.f;
        dvt[d][i] = 0.f;
      }
    const bool ahead = sub == 0 && pre;   // this block prefetches the next one's first tiles
    for (int t = 0; t < nq; ++t) {
      if constexpr (DIAG) d_t0 = stamp_dep(0.f);
      if (t + 1 < nq || ahead) wait_vmcnt<PWV>();   // (younger: tile t+1's or the next block's tile 0)
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      if constexpr (DIAG) {
        const unsigned long long t1 = stamp_dep(0.f);
        d_acc[0] += t1 - d_t0;
        d_t0 = t1;
      }
      const char* lq = smem + cur * BUF;
      const char* ldo_ = lq + TILE;
      const float* ls = reinterpret_cast<const float*>(lq + 2 * TILE);
      const float* ds = ls + 64;
      int nb = cur + 2;
      if (nb >= NST) nb -= NST;
      cur = (cur + 1 == NST) ? 0 : cur + 1;
      const int q0 = qstart + t * BQ;
      if (t + 2 < nq) dma.issue(qbase, dobase, lsb, dlb, ldq, lddo, T, q0 + 2 * BQ, smem + nb * BUF);
      else if (ahead && t + 2 - nq < nq1)   // the next block's tile t + 2 - nq (0 or 1)
        dma.issue(qbase, dobase, lsb, dlb, ldq, lddo, T, qstart1 + (t + 2 - nq) * BQ, smem + nb * BUF);
      if (causal && q0 + BQ - 1 < kw0) {   // wave-uniform: every query of the tile < every key
        if (ahead && t == nq - 1) load_kv(key1);
        continue;
      }
      if constexpr (DIAG) d_acc[7] += 1;
      constexpr int NH = 2 * DTN * 4;
      s16x4 th[(NH + 15) / 16 * 16];
      bf16x8 pd[4];
      // S = Q K^T, dP = dO V^T (rows = queries 32 qt + 8 (i>>2) + 4 hf + (i&3), lane = key).
      // Both row constants are the accumulators' initial values, read from the stage (rows
      // 32 qt + 8 g + 4 hf + 0..3 are 4 consecutive floats): S' = S - lse / scale and
      // dP' = dP - delta, so p = exp2(c2 S') and dS = p dP'.  p of query tile 0 is computed
      // under tile 1's MFMAs (four elements after each pair), tile 1's after them.
      f32x16 sc[2], dp[2];
      // Every LDS read of query tile 0 issued before its first MFMA (row constants, then
      // the Q / dO fragments in MFMA order), tile 1's under tile 0's MFMAs: one LDS latency
      // per half instead of one per MFMA pair
      bf16x8 fa[KS], fb[KS];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 lv = *reinterpret_cast<const f32x4*>(ls + 8 * g + 4 * hf);
        const f32x4 dd = *reinterpret_cast<const f32x4*>(ds + 8 * g + 4 * hf);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sc[0][4 * g + j] = lv[j];
          dp[0][4 * g + j] = dd[j];
        }
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        fa[ks] = *reinterpret_cast<const bf16x8*>(lq + roff[ks]);
        fb[ks] = *reinterpret_cast<const bf16x8*>(ldo_ + roff[ks]);
      }
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 ga[KS], gb[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        sc[0] = MFMA32(fa[ks], kf[ks], sc[0]);
        dp[0] = MFMA32(fb[ks], vf[ks], dp[0]);
        ga[ks] = *reinterpret_cast<const bf16x8*>(lq + roff[ks] + 32 * RB);
        gb[ks] = *reinterpret_cast<const bf16x8*>(ldo_ + roff[ks] + 32 * RB);
        if (ks < 2) {
#pragma unroll
          for (int g = 2 * ks; g < 2 * ks + 2; ++g) {
            const f32x4 lv = *reinterpret_cast<const f32x4*>(ls + 32 + 8 * g + 4 * hf);
            const f32x4 dd = *reinterpret_cast<const f32x4*>(ds + 32 + 8 * g + 4 * hf);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              sc[1][4 * g + j] = lv[j];
              dp[1][4 * g + j] = dd[j];
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        sc[1] = MFMA32(ga[ks], kf[ks], sc[1]);
        dp[1] = MFMA32(gb[ks], vf[ks], dp[1]);
#pragma unroll
        for (int i = (16 / KS) * ks; i < (16 / KS) * (ks + 1); ++i)
          sc[0][i] = __builtin_amdgcn_exp2f(KSC ? sc[0][i] : sc[0][i] * c2);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (DIAG) {
        const unsigned long long t1 = stamp_dep(sc[0][15] + dp[1][15]);
        d_acc[1] += t1 - d_t0;
        d_t0 = t1;
      }
      // dO^T fragments (A of dV^T: lane d = 32 dt + r32, queries 16 s + 4 hf + 0..3 / 8..11)
#pragma unroll
      for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          th[2 * (dt * 4 + s4)] = ds_tr16_off(ldo_ + toff[dt][0], 16 * s4 * RB);
          th[2 * (dt * 4 + s4) + 1] = ds_tr16_off(ldo_ + toff[dt][1], 16 * s4 * RB);
        }
      // dS = p (dP - delta)
      bf16x8 pp[4];
#pragma unroll
      for (int i = 0; i < 16; ++i) sc[1][i] = __builtin_amdgcn_exp2f(KSC ? sc[1][i] : sc[1][i] * c2);
      const bool need_mask = __builtin_amdgcn_readfirstlane(
          (int)((causal && kw0 + 31 > q0) || (q0 + BQ > T) || (kw0 + 32 > T)));
      if (need_mask) {
        // row c = 8 (i>>2) + (i&3) of q-tile qt is query q0 + 32 qt + 4 hf + c: p = 0 when the
        // key is past it (causal: c < key - q0 - 32 qt - 4 hf), or the query / key is >= T
        const int vk = key >= T ? 0x7fffffff : (causal ? key - q0 - 4 * hf : -0x7fffffff);
        const int uq = T - 1 - q0 - 4 * hf;
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int c = 32 * qt + 8 * (i >> 2) + (i & 3);
            sc[qt][i] = (c < vk || c > uq) ? 0.f : sc[qt][i];
          }
      }
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int s1 = 0; s1 < 2; ++s1)
#pragma unroll
          for (int j = 0; j < 8; j += 2) {   // (scalar multiplies: no packed ops beside the MFMAs)
            const int i = 8 * s1 + j;
            pp[2 * qt + s1][j] = (bf16)sc[qt][i];
            pp[2 * qt + s1][j + 1] = (bf16)sc[qt][i + 1];
            pd[2 * qt + s1][j] = (bf16)vmulf(sc[qt][i], dp[qt][i]);
            pd[2 * qt + s1][j + 1] = (bf16)vmulf(sc[qt][i + 1], dp[qt][i + 1]);
          }
      // the block's last tile: K / V are consumed, load the next block's.  Issued here, after
      // every exp / dS of the tile, not between the S / dP MFMAs and the exps: a branch there
      // lets the compiler sink query tile 0's exps below it, out from under tile 1's MFMAs.
      if (ahead && t == nq - 1) load_kv(key1);
      if constexpr (DIAG) {
        const unsigned long long t1 = stamp_dep(__builtin_bit_cast(float, __builtin_bit_cast(u32x4, pd[3])[3]));
        d_acc[2] += t1 - d_t0;
        d_t0 = t1;
      }
#pragma unroll
      for (int w = 0; w < (NH + 15) / 16; ++w) tr_wait8(*reinterpret_cast<s16x4(*)[16]>(&th[16 * w]));
#pragma unroll
      for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          dvt[dt] = MFMA32(tr_join(th[2 * (dt * 4 + s4)], th[2 * (dt * 4 + s4) + 1]), pp[s4], dvt[dt]);
      if constexpr (DIAG) {
        const unsigned long long t1 = stamp_dep(dvt[DTN - 1][15]);
        d_acc[3] += t1 - d_t0;
        d_t0 = t1;
      }
      // Q^T fragments (A of dK^T), read after the dV^T MFMAs are issued
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          th[2 * (dt * 4 + s4)] = ds_tr16_off(lq + toff[dt][0], 16 * s4 * RB);
          th[2 * (dt * 4 + s4) + 1] = ds_tr16_off(lq + toff[dt][1], 16 * s4 * RB);
        }
#pragma unroll
      for (int w = 0; w < (NH + 15) / 16; ++w) tr_wait8(*reinterpret_cast<s16x4(*)[16]>(&th[16 * w]));
#pragma unroll
      for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          dkt[dt] = MFMA32(tr_join(th[2 * (dt * 4 + s4)], th[2 * (dt * 4 + s4) + 1]), pd[s4], dkt[dt]);
      if constexpr (DIAG) d_acc[4] += stamp_dep(dkt[DTN - 1][15]) - d_t0;
    }
    if constexpr (DIAG) d_t0 = stamp_dep(0.f);
    // epilogue: lane = key, registers = d rows 32 dt + 8 g + 4 hf + j.  dK *= scale, inverse
    // RoPE (d pairs with d + HD/2: tile dt with dt + DTN/2, same register), 8-byte stores.  The
    // key's RoPE position is loaded first and dV's row stores and column sums run under that
    // load; then the rotation's table loads and dK's.
    const bool rope = rpos && key < T;
    const int kpos = rope ? reinterpret_cast<const int*>(rpos)[2 * ((long long)b * T + key)] : 0;   // (low word)
    // whole-row stores through the wave's LDS rows (dV, then dK in the same rows: one wave's
    // LDS operations run in order)
    {
      u32x4 rv[RowStage<HD>::NI];
      RowStage<HD>::put(ep, dvt);
      RowStage<HD>::get(ep, rv);
      RowStage<HD>::put_rows(rv, dV + (long long)b * T * lddv + (long long)h * HD, lddv, kw0, T);
    }
    // per-wave column sums over the 32 keys (keys >= T hold zeros): a transpose reduction over
    // the 32 lanes of each half (lane32_sums; the two halves hold disjoint d rows), after which
    // lane r32 holds the sums of registers r32 DTN / 2 + j and stores them
    const long long brow = (((long long)h * (BH / H) + b) * nkb + kb) * 4 + wave;
    if (BPV) {
      float wv[DTN * 16];
#pragma unroll
      for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) wv[16 * dt + i] = key < T ? dvt[dt][i] : 0.f;
      lane32_sums(wv, r32);
#pragma unroll
      for (int j = 0; j < DTN / 2; ++j) {
        const int rr = r32 * (DTN / 2) + j, i = rr & 15;
        BPV[brow * HD + 32 * (rr >> 4) + 8 * (i >> 2) + 4 * hf + (i & 3)] = wv[j];
      }
    }
#pragma unroll
    for (int d = 0; d < DTN; ++d) dkt[d] *= scale;
    if (rope) {
      KASSERT(kpos >= 0, "rope position at key %d", key);
      const float* tr = rtab + (long long)kpos * HD;
#pragma unroll
      for (int dt = 0; dt < DTN / 2; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 cs = *reinterpret_cast<const f32x4*>(tr + 32 * dt + 8 * g + 4 * hf);
          const f32x4 sn = *reinterpret_cast<const f32x4*>(tr + HD / 2 + 32 * dt + 8 * g + 4 * hf);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float x1 = dkt[dt][4 * g + j], x2 = dkt[dt + DTN / 2][4 * g + j];
            dkt[dt][4 * g + j] = x1 * cs[j] + x2 * sn[j];
            dkt[dt + DTN / 2][4 * g + j] = x2 * cs[j] - x1 * sn[j];
          }
        }
    }
    {
      u32x4 rk[RowStage<HD>::NI];
      RowStage<HD>::put(ep, dkt);
      RowStage<HD>::get(ep, rk);
      RowStage<HD>::put_rows(rk, dK + (long long)b * T * lddk + (long long)h * HD, lddk, kw0, T);
    }
    if (BPK) {
      float wk[DTN * 16];
#pragma unroll
      for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) wk[16 * dt + i] = key < T ? dkt[dt][i] : 0.f;
      lane32_sums(wk, r32);
#pragma unroll
      for (int j = 0; j < DTN / 2; ++j) {
        const int rr = r32 * (DTN / 2) + j, i = rr & 15;
        BPK[brow * HD + 32 * (rr >> 4) + 8 * (i >> 2) + 4 * hf + (i & 3)] = wk[j];
      }
    }
    if constexpr (DIAG) d_acc[5] += stamp_dep(0.f) - d_t0;
  }
  if constexpr (DIAG) {
    if (l == 0) {
      unsigned long long* dp = diag + ((long long)blockIdx.x * 4 + wave) * 10;
#pragma unroll
      for (int i = 0; i < 8; ++i) dp[i] = d_acc[i];
      dp[8] = d_start;
      dp[9] = stamp_dep(0.f);
    }
  }
}

// ============================================================================ bwd: dQ ==
// Block: 4 waves x 32 queries = 128 queries; K/V tiles of 64 keys staged in LDS.
template <int HD>
__global__ __launch_bounds__(256, (HD > 64 ? 1 : 2)) void attn_bwd_dq_k(const bf16* __restrict__ Q, const bf16* __restrict__ K,
                                                        const bf16* __restrict__ V, const bf16* __restrict__ dO,
                                                        const bf16* __restrict__ Og, const float* __restrict__ LSE,
                                                        float* __restrict__ DELTA_OUT, float* __restrict__ LSN_OUT,
                                                        bf16* __restrict__ dQ, int T,
                                                        int H, long long ldq, long long ldk, long long ldv,
                                                        long long lddo, long long ldo, long long lddq, float scale,
                                                        int causal, const int64_t* __restrict__ rpos,
                                                        const float* __restrict__ rtab, float* __restrict__ BPQ) {
  // BPQ (optional): each wave's column sums of its stored dQ rows, row ((h * B + b) * nqb +
  // qb) * 4 + wave of a [H * B * nqb * 4, HD] partial (the q bias gradient).
  constexpr int BQ = 128, BKV = 64, KT = HD / 32, DT = HD / 16;
  constexpr int TILE = BKV * HD * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE];
  const int nqb = (T + BQ - 1) / BQ;
  // XCD-aware order: the blocks of one (b, h) -- which share its K / V -- run on one XCD
  // (one L2); within a head the heaviest query blocks still go first.
  const int xl = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
  const int qb = nqb - 1 - xl % gridDim.x;  // heaviest first
  const int bh = xl / gridDim.x, b = bh / H, h = bh % H;
  const int q0 = qb * BQ;
  const int wave = threadIdx.x >> 6, l = lane_id(), g = l >> 4;
  const int wq0 = q0 + wave * 32;
  const float c2 = scale * kLog2e;

  const bf16* kbase = K + (long long)b * T * ldk + (long long)h * HD;
  const bf16* vbase = V + (long long)b * T * ldv + (long long)h * HD;

  bf16x8 qf[2][KT], dof[2][KT];
  float lse2[2], del[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int qi = wq0 + 16 * c + (l & 15);
#pragma unroll
    for (int kk = 0; kk < KT; ++kk) {
      bf16x8 a = {}, d = {};
      if (qi < T) {
        a = *reinterpret_cast<const bf16x8*>(Q + ((long long)b * T + qi) * ldq + (long long)h * HD + 32 * kk + 8 * g);
        d = *reinterpret_cast<const bf16x8*>(dO + ((long long)b * T + qi) * lddo + (long long)h * HD + 32 * kk + 8 * g);
      }
      qf[c][kk] = a;
      dof[c][kk] = d;
    }
    lse2[c] = qi < T ? -LSE[((long long)b * H + h) * T + qi] / scale : 0.f;   // S' = S - lse/scale
    if (g == 0 && qi < T) LSN_OUT[((long long)b * H + h) * T + qi] = lse2[c];
    // delta = rowsum(dO * O), fused here (written for the dK/dV kernel that runs next).
    float dsum = 0.f;
    if (qi < T) {
#pragma unroll
      for (int kk = 0; kk < KT; ++kk) {
        const bf16x8 ov = *reinterpret_cast<const bf16x8*>(Og + ((long long)b * T + qi) * ldo + (long long)h * HD +
                                                           32 * kk + 8 * g);
#pragma unroll
        for (int j = 0; j < 8; ++j) dsum += (float)dof[c][kk][j] * (float)ov[j];
      }
    }
    dsum = group4_sum(dsum);
    del[c] = -dsum;                                                             // dP' = dP - delta
    if (g == 0 && qi < T) DELTA_OUT[((long long)b * H + h) * T + qi] = -dsum;
  }
  f32x4 dq[2][DT];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int d = 0; d < DT; ++d) dq[c][d] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int kv_end = causal ? min(T, q0 + BQ) : T;
  const int nkv = (kv_end + BKV - 1) / BKV;
  Stage<HD, BKV> sk, sv;
  sk.load(kbase, ldk, min(BKV, T));
  sv.load(vbase, ldv, min(BKV, T));
  sk.store(smem);
  sv.store(smem + TILE);
  __syncthreads();

  for (int t = 0; t < nkv; ++t) {
    const int cur = t & 1;
    const char* lk = smem + cur * 2 * TILE;
    const char* lv = lk + TILE;
    const int kv0 = t * BKV;
    const bool more = t + 1 < nkv;
    if (more) {
      const int n0 = kv0 + BKV;
      sk.load(kbase + (long long)n0 * ldk, ldk, min(BKV, T - n0));
      sv.load(vbase + (long long)n0 * ldv, ldv, min(BKV, T - n0));
    }
    const bool wave_active = !causal || kv0 <= wq0 + 31;
    if (wave_active) {
      f32x4 s[4][2], dp[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int c = 0; c < 2; ++c) {   // row constants as initial accumulators (cols = queries)
          s[i][c] = (f32x4){lse2[c], lse2[c], lse2[c], lse2[c]};
          dp[i][c] = (f32x4){del[c], del[c], del[c], del[c]};
        }
      // k-slices outermost: 16 independent MFMAs separate each accumulator's dependent pair
      // (with the slice innermost the compiler padded the chains with ~80 s_nop per tile).
#pragma unroll
      for (int kk = 0; kk < KT; ++kk) {
        bf16x8 kr[4], vr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          kr[i] = row_frag<HD>(lk, 16 * i, 32 * kk);
          vr[i] = row_frag<HD>(lv, 16 * i, 32 * kk);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            s[i][c] = MFMA(kr[i], qf[c][kk], s[i][c]);
            dp[i][c] = MFMA(vr[i], dof[c][kk], dp[i][c]);
          }
      }
      // All 32 S / dP MFMAs issue before the softmax reads their results (interleaved, the
      // scheduler padded each early read with s_nop for the MFMA latency).
      __builtin_amdgcn_sched_barrier(0);
      const bool need_mask = __builtin_amdgcn_readfirstlane(
          (int)((causal && kv0 + BKV - 1 > wq0) || (kv0 + BKV > T)));
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) s[i][c][j] = __builtin_amdgcn_exp2f(s[i][c][j] * c2);
      if (need_mask) {   // wave-uniform: diagonal / tail tiles only, branch-free selects
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int qi = wq0 + 16 * c + (l & 15);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int ki = kv0 + 16 * i + 4 * g + j;
              const bool z = (ki >= T) | (causal & (ki > qi));
              s[i][c][j] = z ? 0.f : s[i][c][j];
            }
        }
      }
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) s[i][c][j] *= dp[i][c][j];  // dS^T
      // dQ^T[d][q] += K^T[d][k] dS^T[k][q]
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 d0 = pack_pt(s[2 * ks][0], s[2 * ks + 1][0]);
        const bf16x8 d1 = pack_pt(s[2 * ks][1], s[2 * ks + 1][1]);
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          const bf16x8 kt = tr_frag<HD>(lk, 32 * ks, 16 * d);
          dq[0][d] = MFMA(kt, d0, dq[0][d]);
          dq[1][d] = MFMA(kt, d1, dq[1][d]);
        }
      }
    }
    if (more) {
      char* nk = smem + (cur ^ 1) * 2 * TILE;
      sk.store(nk);
      sv.store(nk + TILE);
    }
    __syncthreads();
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int qi = wq0 + 16 * c + (l & 15);
    if (qi < T) {
      bf16* row = dQ + ((long long)b * T + qi) * lddq + (long long)h * HD;
#pragma unroll
      for (int d = 0; d < DT; ++d) dq[c][d] *= scale;
      if (rpos) {
        KASSERT(rpos[(long long)b * T + qi] >= 0, "rope position at query %d", qi);
        const float* tr = rtab + rpos[(long long)b * T + qi] * HD;
#pragma unroll
        for (int d = 0; d < DT / 2; ++d) {
          const f32x4 cs = *reinterpret_cast<const f32x4*>(tr + 16 * d + 4 * g);
          const f32x4 sn = *reinterpret_cast<const f32x4*>(tr + HD / 2 + 16 * d + 4 * g);
          const f32x4 x1 = dq[c][d], x2 = dq[c][d + DT / 2];
          dq[c][d] = x1 * cs + x2 * sn;
          dq[c][d + DT / 2] = x2 * cs - x1 * sn;
        }
      }
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        bf16x4 v = {(bf16)dq[c][d][0], (bf16)dq[c][d][1], (bf16)dq[c][d][2], (bf16)dq[c][d][3]};
        *reinterpret_cast<bf16x4*>(row + 16 * d + 4 * g) = v;
      }
    }
  }
  if (BPQ) {
    // Column sums over the wave's 32 queries (2 in-lane, then the 16 lanes of a group).
    f32x4 sq[DT];
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      sq[d] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 2; ++c)
        if (wq0 + 16 * c + (l & 15) < T) sq[d] += dq[c][d];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1)
#pragma unroll
        for (int r = 0; r < 4; ++r) sq[d][r] += __shfl_xor(sq[d][r], o, 64);
    }
    // One partial row per wave (no block barrier: a wave that finishes early leaves).
    if ((l & 15) == 0) {
      float* dst = BPQ + ((((long long)h * (gridDim.y / H) + b) * gridDim.x + qb) * 4 + wave) * HD + 4 * g;
#pragma unroll
      for (int d = 0; d < DT; ++d) *reinterpret_cast<f32x4*>(dst + 16 * d) = sq[d];
    }
  }
}

// ========================================================== bwd: dQ (32x32x16 MFMA) ==
// Query on the lane (as attn_fwd3_k): S^T = K Q^T and dP^T = V dO^T with the keys as the
// 32x32 C rows, so dS^T packed to bf16 is directly the B operand of dQ^T += K^T dS^T (K^T by
// transposed reads of the same K tile).  Also computes delta = rowsum(dO * O) per query and
// writes -lse/scale and -delta for the dK / dV kernel.  K / V tiles (64 keys) by LDS-DMA into
// a 3-slot ring; a workgroup = 4 waves x 32 queries and handles a causal pair of query blocks.
template <int HD>
struct KvDmaU {   // K / V tile rows [kv0, kv0 + 64) into a stage (K at 0, V at TILE), swz_u both
  static constexpr int CPR = HD / 8, TILE = 64 * HD * 2, P = 2 * TILE / 1024, PW = P / 4;
  unsigned voff[PW];
  __device__ __forceinline__ void init(long long ldk, long long ldv) {
    const int l = lane_id(), wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const bool isv = i >= PW / 2;
      const int jj = wave + 4 * i - (isv ? P / 2 : 0);
      const int pos = jj * 64 + l;
      const int r = pos / CPR, cp = pos % CPR;
      voff[i] = (unsigned)(((long long)r * (isv ? ldv : ldk) + swz_u<HD>(r, cp) * 8) * 2);
    }
  }
  __device__ __forceinline__ void issue(const bf16* kb, const bf16* vb, long long ldk, long long ldv, int T, int kv0,
                                        char* stage) const {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(kb + (long long)kv0 * ldk), (short)0, (int)(((long long)(T - 1 - kv0) * ldk + HD) * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(vb + (long long)kv0 * ldv), (short)0, (int)(((long long)(T - 1 - kv0) * ldv + HD) * 2), 0x00020000);
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const bool isv = i >= PW / 2;
      const int jj = wave + 4 * i - (isv ? P / 2 : 0);
      dma16(isv ? rv : rk, stage + (isv ? TILE : 0) + jj * 1024, voff[i]);
    }
  }
};

template <int HD, bool KSC = false>
__global__ __launch_bounds__(256, (HD > 64 ? 1 : 2)) void attn_bwd_dq3_k(
    const bf16* __restrict__ Q, const bf16* __restrict__ K, const bf16* __restrict__ V, const bf16* __restrict__ dO,
    const bf16* __restrict__ Og, const float* __restrict__ LSE, float* __restrict__ NDEL_OUT,
    float* __restrict__ LSN_OUT, bf16* __restrict__ dQ, int T, int H, int BH, long long ldq, long long ldk,
    long long ldv, long long lddo, long long ldo, long long lddq, float scale, int causal,
    const int64_t* __restrict__ rpos, const float* __restrict__ rtab, float* __restrict__ BPQ, int prefetch = 1) {
  static_assert(HD == 64 || HD == 128, "dQ v3: head_dim 64 or 128");
  constexpr int BQ = 128, BKV = 64, KS = HD / 16, DTN = HD / 32, RB = HD * 2;
  constexpr int TILE = BKV * RB, STAGE = 2 * TILE, NST = 3;
  constexpr int PW = KvDmaU<HD>::PW;
  __shared__ __attribute__((aligned(1024))) char smem[NST * STAGE + 4 * RowStage<HD>::BYTES];   // ring, epilogue rows
  const int nqb = (T + BQ - 1) / BQ;
  const int NP = (nqb + 1) / 2;
  const int it = blockIdx.x;
  const int bh = (it >> 3) / NP * 8 + (it & 7), p = (it >> 3) % NP;
  if (bh >= BH) return;
  const int b = bh / H, h = bh % H;
  const int wave = threadIdx.x >> 6, l = lane_id(), r32 = l & 31, hf = l >> 5, g16 = l >> 4, i16 = l & 15;
  char* ep = smem + NST * STAGE + wave * RowStage<HD>::BYTES;
  const float c2 = scale * kLog2e;
  const bf16* kbase = K + (long long)b * T * ldk + (long long)h * HD;
  const bf16* vbase = V + (long long)b * T * ldv + (long long)h * HD;
  KvDmaU<HD> dma;
  dma.init(ldk, ldv);
  int koff[2][KS];   // K / V A-fragment row reads: row 32 kh + r32, chunk 2 ks + hf
#pragma unroll
  for (int kh = 0; kh < 2; ++kh)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int r = 32 * kh + r32;
      koff[kh][ks] = r * RB + (swz_u<HD>(r, 2 * ks + hf) << 4);
    }
  // K^T transposed reads: rows 16 s4 + 4 hf + (i16 >> 2) [+ 8 e], d columns 32 dt + 16 (g16 & 1)
  // + 4 (i16 & 3); swz_u ignores the 16 s4 step (an offset-field immediate), not the + 8
  int toffq[DTN][2];
#pragma unroll
  for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int row = 4 * hf + (i16 >> 2) + 8 * e;
      const int col = 32 * dt + 16 * (g16 & 1) + 4 * (i16 & 3);
      toffq[dt][e] = row * RB + (swz_u<HD>(row, col >> 3) << 4) + (col & 7) * 2;
    }

  // The ring position runs on across the two query blocks (as dK/dV's key blocks): during the
  // first block's last two key tiles the second block's first two K / V tiles are fetched into
  // the slots the first block no longer needs, and its Q / dO / O rows (and LSE) into registers
  // once the last tile's S / dP MFMAs have consumed Q / dO -- the second block starts with its
  // operands landed instead of a cold prologue.  (head_dim 64: at 128 the one-wave-per-SIMD
  // kernel has no registers to spare.)
  const int qb1 = p;
  const int nkv0 = ((causal ? min(T, (nqb - p) * BQ) : T) + BKV - 1) / BKV;
  const int nkv1 = ((causal ? min(T, (qb1 + 1) * BQ) : T) + BKV - 1) / BKV;
  const bool pre = HD == 64 && (prefetch & 1) && qb1 != nqb - 1 - p && nkv0 >= 2 && nkv1 > 0;   // (uniform)
  for (int sn = 0; sn < (blockIdx.x & 1) * (prefetch >> 4); ++sn) __builtin_amdgcn_s_sleep(127);
  bf16x8 qf[KS], df[KS], ovr[KS];   // Q^T / dO^T operands (lane: query), O for delta
  float lse_r = 0.f;
  auto load_qdo = [&](int qq) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 a = {}, c = {}, ov = {};
      if (qq < T) {
        a = *reinterpret_cast<const bf16x8*>(Q + ((long long)b * T + qq) * ldq + (long long)h * HD + 16 * ks + 8 * hf);
        c = *reinterpret_cast<const bf16x8*>(dO + ((long long)b * T + qq) * lddo + (long long)h * HD + 16 * ks + 8 * hf);
        ov = *reinterpret_cast<const bf16x8*>(Og + ((long long)b * T + qq) * ldo + (long long)h * HD + 16 * ks + 8 * hf);
      }
      qf[ks] = a;
      df[ks] = c;
      ovr[ks] = ov;
    }
    lse_r = qq < T ? LSE[(long long)bh * T + qq] : 0.f;
  };
  int cur = 0;
  for (int sub = 0; sub < 2; ++sub) {
    const int qb = sub == 0 ? nqb - 1 - p : p;
    if (sub == 1 && qb == nqb - 1 - p) break;
    if (sub == 1) __syncthreads();
    const int q0 = qb * BQ, wq0 = q0 + 32 * wave, qi = wq0 + r32;
    // the query's RoPE position (low word of the int64), loaded with the block's prologue
    const int qpos = (rpos && qi < T) ? reinterpret_cast<const int*>(rpos)[2 * ((long long)b * T + qi)] : 0;
    const int kv_end = causal ? min(T, q0 + BQ) : T;
    const int nkv = (kv_end + BKV - 1) / BKV;
    const bool fetched = sub == 1 && pre;   // tiles 0 / 1 and the Q / dO / O rows already on their way
    if (!fetched) {
      const int c1 = cur + 1 == NST ? 0 : cur + 1;
      dma.issue(kbase, vbase, ldk, ldv, T, 0, smem + cur * STAGE);
      if (nkv > 1) dma.issue(kbase, vbase, ldk, ldv, T, BKV, smem + c1 * STAGE);
      // Q^T / dO^T operands (B of S^T, dP^T): lane holds X[qi][16 ks + 8 hf + j]
      load_qdo(qi);
    }
    wait_vmcnt<0>();
    asm volatile("" ::"v"(qpos));   // (keeps the position load here, not sunk to its use)
    float dsum = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) dsum += (float)df[ks][j] * (float)ovr[ks][j];
    const float lc = qi < T ? -lse_r * kLog2e : 0.f;   // p = exp2(c2 S + lc)
    const float ndel = -pair_sum(dsum);                                      // dP' = dP - delta
    if (hf == 0 && qi < T) {
      // dK/dV: S' = S - lse / scale (KSC: S' = S scale log2 e - lse log2 e, K pre-scaled)
      LSN_OUT[(long long)bh * T + qi] = KSC ? -lse_r * kLog2e : -lse_r / scale;
      NDEL_OUT[(long long)bh * T + qi] = ndel;
    }
    f32x16 dq[DTN];
#pragma unroll
    for (int d = 0; d < DTN; ++d)
#pragma unroll
      for (int i = 0; i < 16; ++i) dq[d][i] = 0.f;
    const bool ahead = sub == 0 && pre;   // this block prefetches the next one's first tiles
    const int qi1 = qb1 * BQ + 32 * wave + r32;
    for (int t = 0; t < nkv; ++t) {
      if (t + 1 < nkv || ahead) wait_vmcnt<PW>();   // (younger: tile t+1's or the next block's tile 0)
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      const char* lk = smem + cur * STAGE;
      const char* lv = lk + TILE;
      int nb = cur + 2;
      if (nb >= NST) nb -= NST;
      cur = (cur + 1 == NST) ? 0 : cur + 1;
      const int kv0 = t * BKV;
      if (t + 2 < nkv) dma.issue(kbase, vbase, ldk, ldv, T, kv0 + 2 * BKV, smem + nb * STAGE);
      else if (ahead && t + 2 - nkv < nkv1)   // the next block's tile t + 2 - nkv (0 or 1)
        dma.issue(kbase, vbase, ldk, ldv, T, (t + 2 - nkv) * BKV, smem + nb * STAGE);
      if (causal && kv0 > wq0 + 31) {   // wave-uniform
        if (ahead && t == nkv - 1) load_qdo(qi1);
        continue;
      }
      // dP^T starts from -delta (the lane's query), so dS = p dP' directly; p of key half 0 is
      // computed under half 1's MFMAs (four elements after each pair), half 1's after them.
      f32x16 sc[2], dp[2];
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          sc[kh][i] = 0.f;
          dp[kh][i] = ndel;
        }
      // Key half 0's K / V fragments all read before its first MFMA, half 1's under
      // half 0's MFMAs (one LDS latency per half instead of one per MFMA pair)
      bf16x8 fa[KS], fb[KS], ga[KS], gb[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        fa[ks] = *reinterpret_cast<const bf16x8*>(lk + koff[0][ks]);
        fb[ks] = *reinterpret_cast<const bf16x8*>(lv + koff[0][ks]);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        sc[0] = MFMA32(fa[ks], qf[ks], sc[0]);
        dp[0] = MFMA32(fb[ks], df[ks], dp[0]);
        ga[ks] = *reinterpret_cast<const bf16x8*>(lk + koff[1][ks]);
        gb[ks] = *reinterpret_cast<const bf16x8*>(lv + koff[1][ks]);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        sc[1] = MFMA32(ga[ks], qf[ks], sc[1]);
        dp[1] = MFMA32(gb[ks], df[ks], dp[1]);
#pragma unroll
        for (int i = (16 / KS) * ks; i < (16 / KS) * (ks + 1); ++i)
          sc[0][i] = __builtin_amdgcn_exp2f(fmaf(sc[0][i], c2, lc));
        __builtin_amdgcn_sched_barrier(0);
      }
      // K^T fragments (A of dQ^T: lane d = 32 dt + r32, keys 16 s + 4 hf + 0..3 / 8..11)
      constexpr int NH = 2 * DTN * 4;
      s16x4 th[(NH + 15) / 16 * 16];
#pragma unroll
      for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          th[2 * (dt * 4 + s4)] = ds_tr16_off(lk + toffq[dt][0], 16 * s4 * RB);
          th[2 * (dt * 4 + s4) + 1] = ds_tr16_off(lk + toffq[dt][1], 16 * s4 * RB);
        }
#pragma unroll
      for (int i = 0; i < 16; ++i) sc[1][i] = __builtin_amdgcn_exp2f(fmaf(sc[1][i], c2, lc));
      const bool need_mask = __builtin_amdgcn_readfirstlane(
          (int)((causal && kv0 + BKV - 1 > wq0) || (kv0 + BKV > T)));
      if (need_mask) {
        const int lim = (causal ? min(qi, T - 1) : T - 1) - kv0 - 4 * hf;
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            sc[kh][i] = (32 * kh + 8 * (i >> 2) + (i & 3) > lim) ? 0.f : sc[kh][i];
      }
      bf16x8 pd[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int j = 0; j < 8; j += 2) {   // (scalar multiplies: no packed ops beside the MFMAs)
          const int kh = s4 >> 1, i = 8 * (s4 & 1) + j;
          pd[s4][j] = (bf16)vmulf(sc[kh][i], dp[kh][i]);
          pd[s4][j + 1] = (bf16)vmulf(sc[kh][i + 1], dp[kh][i + 1]);
        }
      // the block's last tile: Q / dO are consumed, load the next block's rows (after the exps
      // and dS: a branch between the S / dP MFMAs and the exps lets the compiler sink key half
      // 0's exps out from under half 1's MFMAs)
      if (ahead && t == nkv - 1) load_qdo(qi1);
#pragma unroll
      for (int w = 0; w < (NH + 15) / 16; ++w) tr_wait8(*reinterpret_cast<s16x4(*)[16]>(&th[16 * w]));
#pragma unroll
      for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          dq[dt] = MFMA32(tr_join(th[2 * (dt * 4 + s4)], th[2 * (dt * 4 + s4) + 1]), pd[s4], dq[dt]);
    }
    // epilogue: lane = query, registers = d rows 32 dt + 8 g + 4 hf + j: scale, inverse RoPE
#pragma unroll
    for (int d = 0; d < DTN; ++d) dq[d] *= scale;
    if (rpos && qi < T) {
      KASSERT(qpos >= 0, "rope position at query %d", qi);
      const float* tr = rtab + (long long)qpos * HD;
#pragma unroll
      for (int dt = 0; dt < DTN / 2; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 cs = *reinterpret_cast<const f32x4*>(tr + 32 * dt + 8 * g + 4 * hf);
          const f32x4 sn = *reinterpret_cast<const f32x4*>(tr + HD / 2 + 32 * dt + 8 * g + 4 * hf);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float x1 = dq[dt][4 * g + j], x2 = dq[dt + DTN / 2][4 * g + j];
            dq[dt][4 * g + j] = x1 * cs[j] + x2 * sn[j];
            dq[dt + DTN / 2][4 * g + j] = x2 * cs[j] - x1 * sn[j];
          }
        }
    }
    {   // whole-row stores through the wave's LDS rows
      u32x4 rq[RowStage<HD>::NI];
      RowStage<HD>::put(ep, dq);
      RowStage<HD>::get(ep, rq);
      RowStage<HD>::put_rows(rq, dQ + (long long)b * T * lddq + (long long)h * HD, lddq, wq0, T);
    }
    if (BPQ) {   // per-wave column sums over the 32 queries (lane32_sums, as dK / dV's)
      const long long prow = (((long long)h * (BH / H) + b) * nqb + qb) * 4 + wave;
      float wq[DTN * 16];
#pragma unroll
      for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) wq[16 * dt + i] = qi < T ? dq[dt][i] : 0.f;
      lane32_sums(wq, r32);
#pragma unroll
      for (int j = 0; j < DTN / 2; ++j) {
        const int rr = r32 * (DTN / 2) + j, i = rr & 15;
        BPQ[prow * HD + 32 * (rr >> 4) + 8 * (i >> 2) + 4 * hf + (i & 3)] = wq[j];
      }
    }
  }
}

}  // namespace dpfs

using namespace dpfs;

#define HD_DISPATCH(HDV, ...)                           \
  do {                                                       \
    if ((HDV) == 64) { constexpr int HD_ = 64; __VA_ARGS__; } \
    else if ((HDV) == 128) { constexpr int HD_ = 128; __VA_ARGS__; } \
    else if ((HDV) == 32) { constexpr int HD_ = 32; __VA_ARGS__; } \
  } while (0)

extern "C" int dpfs_attn_supported_hd(int hd) { return hd == 32 || hd == 64 || hd == 128; }

// Kernel selection is a per-call argument (`impl`), never process state.
// Forward: 0 = auto (attn_fwd3_k at head_dim 64 / 128, attn_fwd_k otherwise), 1 = attn_fwd_k
// (16x16x32, register-staged), 4 = attn_fwd3_k (32x32x16, LDS-DMA ring, hd 64 / 128), 5 = its
// DIAG build (hd 64, timing diagnosis into the attn_diag buffer).  (Round 4 retired impl 2 / 3,
// the 16x16x32 LDS-DMA forward: slower than impl 4 at every head_dim it supported.)
// The DIAG builds' output buffer (tools/attn_probe.py --diag) is the one piece of state: it is
// read only by a call that asks for a DIAG build.
static unsigned long long* g_attn_diag = nullptr;
extern "C" void dpfs_attn_diag(void* p) { g_attn_diag = (unsigned long long*)p; }
// dK/dV (head_dim 64): 1 = the second key block's first tiles / K / V fetched during the first
// block's last tiles (default), 0 = a cold prologue per block (A/B probes)
// Cross-block operand prefetch of the head_dim-64 backward kernels (A/B hook): bit 0 = dK/dV,
// bit 1 = dQ (3 default)
static int g_attn_prefetch = 3;
extern "C" void dpfs_attn_prefetch(int v) { g_attn_prefetch = v & 3; }
// A/B hook: odd workgroups of the v3 backward kernels start v x 8k cycles late (0 default)
static int g_attn_stagger = 0;
extern "C" void dpfs_attn_stagger(int v) { g_attn_stagger = v & 15; }

extern "C" void dpfs_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int T, int H,
                              int hd, long long ldq, long long ldk, long long ldv, long long ldo, float scale,
                              int causal, int impl_req, hipStream_t s) {
  const int impl = impl_req == 0 ? ((hd == 64 || hd == 128) ? 4 : 1) : impl_req;
  if (impl == 8 && (hd == 64 || hd == 128)) {   // scale and max folded into the MFMAs (A/B)
    const int nqb = (T + 127) / 128, grid = (B * H + 7) / 8 * 8 * ((nqb + 1) / 2);
    if (hd == 64)
      attn_fwd3_k<64, 0, false, true><<<grid, 256, 0, s>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o,
                                                           lse, T, H, B * H, ldq, ldk, ldv, ldo, scale, causal);
    else
      attn_fwd3_k<128, 0, false, true><<<grid, 256, 0, s>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o,
                                                            lse, T, H, B * H, ldq, ldk, ldv, ldo, scale, causal);
    return;
  }
  if (impl == 6 && (hd == 64 || hd == 128)) {   // the row sum by MFMA (A/B)
    const int nqb = (T + 127) / 128, grid = (B * H + 7) / 8 * 8 * ((nqb + 1) / 2);
    if (hd == 64)
      attn_fwd3_k<64, 0, true><<<grid, 256, 0, s>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, lse, T,
                                                    H, B * H, ldq, ldk, ldv, ldo, scale, causal);
    else
      attn_fwd3_k<128, 0, true><<<grid, 256, 0, s>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, lse,
                                                     T, H, B * H, ldq, ldk, ldv, ldo, scale, causal);
    return;
  }
  if ((impl == 4 || (impl == 5 && g_attn_diag)) && (hd == 64 || hd == 128)) {
    // one workgroup per item (the dispatcher refills freed slots, which balances the end of
    // the kernel; a persistent grid measured slower)
    const int nqb = (T + 127) / 128, grid = (B * H + 7) / 8 * 8 * ((nqb + 1) / 2);
    if (hd == 64 && impl == 5)
      attn_fwd3_k<64, 1><<<grid, 256, 0, s>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, lse, T, H,
                                              B * H, ldq, ldk, ldv, ldo, scale, causal, g_attn_diag);
    else if (hd == 64)
      attn_fwd3_k<64><<<grid, 256, 0, s>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, lse, T, H,
                                           B * H, ldq, ldk, ldv, ldo, scale, causal);
    else
      attn_fwd3_k<128><<<grid, 256, 0, s>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, lse, T, H,
                                            B * H, ldq, ldk, ldv, ldo, scale, causal);
    return;
  }
  dim3 grid((T + 127) / 128, B * H);
  HD_DISPATCH(hd, attn_fwd_k<HD_><<<grid, 256, 0, s>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o,
                                                            lse, T, H, ldq, ldk, ldv, ldo, scale, causal));
}

// attention_fused.hip (its own translation unit: asm-owned AGPR accumulators)
extern "C" void dpfs_attn_bwd_dkdv4(int items, const void* q, const void* k, const void* v, const void* dout,
                                    const float* lsn, const float* ndel, void* dk, void* dv, int T, int H, int BH,
                                    long long ldq, long long ldk, long long ldv, long long lddo, long long lddk,
                                    long long lddv, float scale, int causal, const int64_t* rope_pos,
                                    const float* rope_tab, float* pk, float* pv, int prefetch, hipStream_t s);

// delta: workspace [2][B, H, T] fp32: -delta (rowsum(dO*O)) and -lse/scale, written by the dQ kernel.
// Backward kernel pair (`impl`): 0 = auto (4 at head_dim 64 / 128, 2 otherwise), 2 =
// attn_bwd_dq_k + attn_bwd_dkdv2_k (16x16x32, LDS-DMA ring), 4 = attn_bwd_dq3_k +
// attn_bwd_dkdv3_k (32x32x16, query / key on the lane, hd 64 / 128), 5 = 4 with the dK/dV DIAG
// build (hd 64, into the attn_diag buffer).  (Round 4 retired the register-staged dK/dV
// kernels, impl 1 / 3.)
extern "C" int dpfs_attn_bwd(const void* dout, const void* q, const void* k, const void* v, const void* o,
                              const float* lse, float* delta, void* dq, void* dk, void* dv, int B, int T, int H,
                              int hd, long long lddo, long long ldq, long long ldk, long long ldv, long long ldo,
                              long long lddq, long long lddk, long long lddv, float scale, int causal,
                              const int64_t* rope_pos, const float* rope_tab, hipStream_t s, float* dbias,
                              float* bws, int impl_req) {
  // The QKV bias gradient rides on both kernel pairs' epilogues (per-wave column sums + one
  // reduction kernel).
  const bool v3ok = hd == 64 || hd == 128;
  const bool diag = impl_req == 5 && g_attn_diag != nullptr;
  // 7 = attn_bwd_dq3_k + attn_bwd_dkdv4_k (64 keys per wave, head_dim 64; else 4)
  const bool v4 = impl_req == 7 && hd == 64;
  // 9 = impl 4 with the K pre-scale (KSC, A/B; the 64-keys-per-wave dK/dV of impl 7 uses it too)
  const bool ksc = impl_req == 9 || impl_req == 7;
  const int bimpl = impl_req == 0 ? (v3ok ? 4 : 2) : ((impl_req == 5 || impl_req == 7 || impl_req == 9) ? 4 : impl_req);
  const bool bias = dbias != nullptr && bws != nullptr;
  const int nqb = (T + 127) / 128, nkb = (T + 63) / 64;
  float* pq = bias ? bws : nullptr;
  float* pk = bias ? bws + (long long)H * B * nqb * 4 * hd : nullptr;
  float* pv = bias ? pk + (long long)H * B * nkb * 4 * hd : nullptr;
  dim3 gq(nqb, B * H);
  if (bimpl == 4 && v3ok) {   // (attn_bwd_dkdv3_k reads the -lse / scale this kernel writes)
    const int items = (B * H + 7) / 8 * 8 * ((nqb + 1) / 2);
#define DQ3_LAUNCH(HD_)                                                                                             \
  do { if (ksc) attn_bwd_dq3_k<HD_, true><<<items, 256, 0, s>>>(                                                         \
      (const bf16*)q, (const bf16*)k, (const bf16*)v, (const bf16*)dout, (const bf16*)o, lse, delta,                \
      delta + (long long)B * H * T, (bf16*)dq, T, H, B * H, ldq, ldk, ldv, lddo, ldo, lddq, scale, causal, rope_pos,  \
      rope_tab, pq, ((g_attn_prefetch >> 1) & 1) | (g_attn_stagger << 4));                                           \
  else attn_bwd_dq3_k<HD_, false><<<items, 256, 0, s>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (const bf16*)dout,   \
                                            (const bf16*)o, lse, delta, delta + (long long)B * H * T, (bf16*)dq, T, \
                                            H, B * H, ldq, ldk, ldv, lddo, ldo, lddq, scale, causal, rope_pos,     \
                                            rope_tab, pq, ((g_attn_prefetch >> 1) & 1) | (g_attn_stagger << 4)); } while (0)
    if (hd == 64) DQ3_LAUNCH(64);
    else DQ3_LAUNCH(128);
#undef DQ3_LAUNCH
  } else
  HD_DISPATCH(hd, attn_bwd_dq_k<HD_><<<gq, 256, 0, s>>>((const bf16*)q, (const bf16*)k, (const bf16*)v,
                                                             (const bf16*)dout, (const bf16*)o, lse, delta,
                                                             delta + (long long)B * H * T, (bf16*)dq,
                                                             T, H, ldq, ldk, ldv, lddo, ldo, lddq, scale, causal,
                                                             rope_pos, rope_tab, pq));
  if (bimpl == 4 && v3ok) {
    const int nkb3 = (T + 127) / 128, items = (B * H + 7) / 8 * 8 * ((nkb3 + 1) / 2);
    const int nkb4 = (T + 255) / 256, items4 = (B * H + 7) / 8 * 8 * ((nkb4 + 1) / 2);
    if (v4)
      dpfs_attn_bwd_dkdv4(items4, q, k, v, dout, delta + (long long)B * H * T, delta, dk, dv, T, H, B * H, ldq, ldk,
                          ldv, lddo, lddk, lddv, scale, causal, rope_pos, rope_tab, pk, pv, g_attn_prefetch & 1, s);
    else {
#define DKDV3_LAUNCH(HD_, DG_)                                                                                      \
  do { if (ksc) attn_bwd_dkdv3_k<HD_, DG_, true><<<items, 256, 0, s>>>((const bf16*)q, (const bf16*)k, (const bf16*)v,       \
      (const bf16*)dout, delta + (long long)B * H * T, delta, (bf16*)dk, (bf16*)dv, T, H, B * H, ldq, ldk, ldv, lddo,  \
      lddk, lddv, scale, causal, rope_pos, rope_tab, pk, pv, DG_ ? g_attn_diag : nullptr,                              \
      (g_attn_prefetch & 1) | (g_attn_stagger << 4));                                                                  \
  else attn_bwd_dkdv3_k<HD_, DG_, false><<<items, 256, 0, s>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (const bf16*)dout, \
                                                   delta + (long long)B * H * T, delta, (bf16*)dk, (bf16*)dv, T, H,     \
                                                   B * H, ldq, ldk, ldv, lddo, lddk, lddv, scale, causal, rope_pos,     \
                                                   rope_tab, pk, pv, DG_ ? g_attn_diag : nullptr, (g_attn_prefetch & 1) | (g_attn_stagger << 4)); } while (0)
    if (hd == 64 && diag) DKDV3_LAUNCH(64, 1);
    else if (hd == 64) DKDV3_LAUNCH(64, 0);
    else DKDV3_LAUNCH(128, 0);
#undef DKDV3_LAUNCH
    }
    if (bias) {
      if (hd == 64) attn_bias_grad_k<64><<<3 * H * 4, 1024, 0, s>>>(pq, pk, pv, dbias, H, B * nqb * 4, B * nkb3 * 4);
      else attn_bias_grad_k<128><<<3 * H * 8, 1024, 0, s>>>(pq, pk, pv, dbias, H, B * nqb * 4, B * nkb3 * 4);
      return 1;
    }
    return 0;
  }
  dim3 gk((T + 63) / 64, B * H);
  HD_DISPATCH(hd, attn_bwd_dkdv2_k<HD_><<<gk, 256, 0, s>>>((const bf16*)q, (const bf16*)k, (const bf16*)v,
                                                                (const bf16*)dout, delta + (long long)B * H * T,
                                                                delta, (bf16*)dk,
                                                                (bf16*)dv, T, H, ldq, ldk, ldv, lddo, lddk, lddv,
                                                                scale, causal, rope_pos, rope_tab, pk, pv));
  if (bias) {
    HD_DISPATCH(hd, attn_bias_grad_k<HD_><<<3 * H * (HD_ / 16), 1024, 0, s>>>(pq, pk, pv, dbias, H,
                                                                                     B * nqb * 4, B * nkb * 4));
    return 1;
  }
  return 0;
}

// Floats of the bias-gradient partials dpfs_attn_bwd needs (one q row per dQ wave, one k and
// one v row per dK/dV wave, HD columns each).
extern "C" long long dpfs_attn_bias_ws(int B, int T, int H, int hd) {
  const long long nqb = (T + 127) / 128, nkb = (T + 63) / 64;
  return (long long)H * B * (nqb + 2 * nkb) * 4 * hd;
}
