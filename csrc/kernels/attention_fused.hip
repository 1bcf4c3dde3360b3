// Fused attention backward for head_dim 64 (impl 6 of dpfs_attn_bwd): see the comment block
// below.  Its own translation unit: built with -mllvm -amdgpu-mfma-vgpr-form (tools/build_ext.py)
// so the compiler keeps its MFMA accumulators in VGPRs; the long-lived dK^T / dV^T
// accumulators live in asm-owned AGPRs.
#include "attn_common.h"

namespace dpfs {

#include "attn_acc.inc"

// run-time block index (constant after unrolling: the switch folds)
__device__ __forceinline__ void acc32_mfma_i(int i, const bf16x8& a, const bf16x8& b) {
  switch (i) {
    case 0: acc32_mfma<0>(a, b); break;
    case 1: acc32_mfma<1>(a, b); break;
    case 2: acc32_mfma<2>(a, b); break;
    case 3: acc32_mfma<3>(a, b); break;
    case 4: acc32_mfma<4>(a, b); break;
    case 5: acc32_mfma<5>(a, b); break;
    case 6: acc32_mfma<6>(a, b); break;
    default: acc32_mfma<7>(a, b); break;
  }
}

// ================================================ bwd: fused dK / dV / dQ (head_dim 64) ==
// One pass over the causal (key block x query tile) pairs computes all five backward products
// (S = Q K^T, dP = dO V^T, dV^T += dO^T P, dK^T += Q^T dS, dQ^T += K^T dS^T) instead of the
// dQ + dK/dV kernel pair's seven (both of which recompute S and dP).  Guide §B 'Attention
// backward' structure at head_dim 64:
//  * workgroup = 4 waves = 256 keys of one (b, h), ONE wave per SIMD (512 registers): wave w
//    owns keys 64 w .. 64 w + 63 and keeps their dK^T / dV^T (128 accumulator registers) and
//    K / V B operands (64) for the whole query sweep; a causal pair of key blocks (p, nkb-1-p)
//    per workgroup gives every workgroup the same work.
//  * query tiles of 64 rows (Q, dO, -lse/scale, -delta) stream through the 3-slot LDS-DMA ring
//    of the v3 kernels (QdoDma3, swz_u); each Q / dO fragment read feeds both 32-key halves.
//  * dS leaves each wave once, as bf16 [key][query] rows in LDS (swz_u: conflict-free for the
//    8-byte row writes and the transposed reads); after the next tile's barrier every wave
//    computes one 32 x 32 (d x query) block of dQ^T over all 256 keys from it (K^T fragments
//    held in registers), so dQ leaves the workgroup already summed over its keys, as a
//    deterministic fp32 partial (plain stores, no atomics) that attn_dq_reduce_k adds up
//    over the key blocks in a fixed order.
//  * software pipeline per tile, over the four (query half, key half) blocks j: S / dP of j,
//    the softmax-gradient VALU of j - 1 and the dV / dK MFMAs of j - 2 (and the previous
//    tile's dQ) share each stretch of MFMAs, so the exponentials issue beside matrix work.
// The row constants (-delta, -lse/scale) come from attn_bwd_delta_k.

// delta = rowsum(dO * O) and the dK/dV row constants: NDEL = -delta, LSN = -lse / scale, both
// (B, H, T) fp32.  HD / 8 lanes per (b, t, h) row, one 16-byte load of dO and O each.
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_delta_k(const bf16* __restrict__ dO, const bf16* __restrict__ Og,
                                                        const float* __restrict__ LSE, float* __restrict__ NDEL,
                                                        float* __restrict__ LSN, int T, int H, long long rows,
                                                        long long lddo, long long ldo, float inv_scale) {
  constexpr int TPR = HD / 8;
  const long long gt = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long row = gt / TPR;
  const int c = (int)(gt % TPR);
  float s = 0.f;
  const bool ok = row < rows;
  const int h = ok ? (int)(row % H) : 0;
  const long long bt = ok ? row / H : 0;
  if (ok) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(dO + bt * lddo + (long long)h * HD + 8 * c);
    const bf16x8 o = *reinterpret_cast<const bf16x8*>(Og + bt * ldo + (long long)h * HD + 8 * c);
#pragma unroll
    for (int j = 0; j < 8; ++j) s = fmaf((float)a[j], (float)o[j], s);
  }
#pragma unroll
  for (int o = TPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (ok && c == 0) {
    const long long b = bt / T, t = bt % T;
    const long long idx = (b * H + h) * T + t;
    NDEL[idx] = -s;
    LSN[idx] = -LSE[idx] * inv_scale;
  }
}

__device__ __forceinline__ void ds_write64(const char* p, u32x2 v) {
  asm volatile("ds_write_b64 %0, %1" ::"v"(lds_u32(p)), "v"(v));
}

// fp32 dQ partial of one (b, h, key block, query tile): 4 waves x 1024 floats, each wave's
// 32 x 32 (query x d) block in accumulator order: float (g * 64 + lane) * 4 + j holds register
// 4 g + j of lane `lane` (query 32 (w >> 1) + (lane & 31), d 32 (w & 1) + 8 g + 4 (lane >> 5) + j).
constexpr int kDqChunk = 4096;

template <int HD>
__global__ __launch_bounds__(256, 1) void attn_bwd_fused_k(
    const bf16* __restrict__ Q, const bf16* __restrict__ K, const bf16* __restrict__ V, const bf16* __restrict__ dO,
    const float* __restrict__ LSN, const float* __restrict__ NDEL, bf16* __restrict__ dK, bf16* __restrict__ dV,
    float* __restrict__ DQP, int T, int H, int BH, long long ldq, long long ldk, long long ldv, long long lddo,
    long long lddk, long long lddv, float scale, int causal, const int64_t* __restrict__ rpos,
    const float* __restrict__ rtab, float* __restrict__ BPK, float* __restrict__ BPV) {
  static_assert(HD == 64, "fused backward: head_dim 64");
  constexpr int KB = 256, BQ = 64, KS = HD / 16, DTN = HD / 32, RB = HD * 2;
  constexpr int TILE = BQ * RB, BUF = 2 * TILE + 1024, NST = 3;
  constexpr int DSB = KB * BQ * 2;                    // one dS buffer: [256 keys][64 queries] bf16
  constexpr int PWV = QdoDma3<HD>::PW + 1;            // DMA instructions per wave per tile
  constexpr int NSTORE = 4;                           // dQ partial stores per wave per tile
  // [ring | dS 0 | dS 1 | K rows of the key block]; the epilogue rows reuse the (idle) ring
  __shared__ __attribute__((aligned(1024))) char smem[NST * BUF + 3 * DSB];
  static_assert(4 * RowStage<HD>::BYTES <= NST * BUF, "epilogue rows fit the ring");
  const int nkb = (T + KB - 1) / KB, nqt = (T + BQ - 1) / BQ;
  const int NP = (nkb + 1) / 2;
  const int it = blockIdx.x;
  const int bh = (it >> 3) / NP * 8 + (it & 7), p = (it >> 3) % NP;
  if (bh >= BH) return;
  const int b = bh / H, h = bh % H;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l = lane_id(), r32 = l & 31, hf = l >> 5, g16 = l >> 4, i16 = l & 15;
  char* const dsb = smem + NST * BUF;
  const char* const kst = dsb + 2 * DSB;
  char* const ep = smem + wave * RowStage<HD>::BYTES;
  const float c2 = scale * kLog2e;
  const bf16* qbase = Q + (long long)b * T * ldq + (long long)h * HD;
  const bf16* dobase = dO + (long long)b * T * lddo + (long long)h * HD;
  const float* lsb = LSN + (long long)bh * T;
  const float* dlb = NDEL + (long long)bh * T;
  QdoDma3<HD> dma;
  dma.init(ldq, lddo);
  const int dqt = wave >> 1, ddt = wave & 1;   // this wave's dQ^T block: queries 32 dqt.., d 32 ddt..
  // lane-constant LDS offsets (swz_u tiles of 128-byte rows; + 16-row steps and + 32-row steps
  // keep the swizzle, so they ride the instructions' offset fields):
  //  roff: Q / dO row fragments (row r32, chunk 2 ks + hf)
  //  toff: transposed fragments, rows 4 hf + (i16 >> 2) [+ 8 e], columns 32 c + 16 (g16 & 1) +
  //        4 (i16 & 3): dO^T / Q^T (c = dt), dS^T (c = dqt) and K^T (c = ddt)
  int roff[KS], toff[DTN][2], doff[2], koff[2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) roff[ks] = r32 * RB + (swz_u<HD>(r32, 2 * ks + hf) << 4);
  auto tro = [&](int e, int c) {
    const int row = 4 * hf + (i16 >> 2) + 8 * e;
    const int col = 32 * c + 16 * (g16 & 1) + 4 * (i16 & 3);
    return row * RB + (swz_u<HD>(row, col >> 3) << 4) + (col & 7) * 2;
  };
#pragma unroll
  for (int e = 0; e < 2; ++e) {
#pragma unroll
    for (int dt = 0; dt < DTN; ++dt) toff[dt][e] = tro(e, dt);
    doff[e] = tro(e, dqt);
    koff[e] = tro(e, ddt);
  }
  // dS row writes: key row 64 wave + 32 kh + r32, query columns 32 qt + 8 g + 4 hf + 0..3: the
  // 16-byte chunk 4 qt + g of that row, XORed by the row's swizzle (a function of r32 only)
  const int wrow = (64 * wave + r32) * RB + 8 * hf;
  const int wsw = swz_u<HD>(r32, 0);

  const int kb1 = nkb - 1 - p;
  for (int sub = 0; sub < 2; ++sub) {
    const int kb = sub == 0 ? p : kb1;
    if (sub == 1 && kb == p) break;
    __syncthreads();   // (sub 1) the previous key block's dS / ring / epilogue reads are done
    const int k0 = kb * KB, kw0 = k0 + 64 * wave;
    const int qstart = causal ? k0 : 0;   // k0 is a multiple of BQ
    const int nq = (T - qstart + BQ - 1) / BQ;
    const int qt0 = qstart / BQ;
    int cur = 0;
    if (nq > 0) dma.issue(qbase, dobase, lsb, dlb, ldq, lddo, T, qstart, smem);
    if (nq > 1) dma.issue(qbase, dobase, lsb, dlb, ldq, lddo, T, qstart + BQ, smem + BUF);
    // K / V B operands of S / dP (lane: key 32 kh + r32; d 16 ks + 8 hf + 0..7) in registers
    bf16x8 kf[2][KS], vf[2][KS];
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int key = kw0 + 32 * kh + r32;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8 a_ = {}, c_ = {};
        if (key < T) {
          a_ = *reinterpret_cast<const bf16x8*>(K + ((long long)b * T + key) * ldk + (long long)h * HD + 16 * ks + 8 * hf);
          c_ = *reinterpret_cast<const bf16x8*>(V + ((long long)b * T + key) * ldv + (long long)h * HD + 16 * ks + 8 * hf);
        }
        kf[kh][ks] = a_;
        vf[kh][ks] = c_;
      }
    }
    // the block's 256 K rows into LDS (swz_u rows): K^T fragments of this wave's d half are
    // the A operands of dQ^T (transposed reads, keys 16 s + 4 hf + 0..3 / 8..11)
    {
      char* kw = dsb + 2 * DSB;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = threadIdx.x + 256 * i, row = c >> 3, ch = c & 7;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (k0 + row < T)
          v = *reinterpret_cast<const u32x4*>(K + ((long long)b * T + k0 + row) * ldk + (long long)h * HD + ch * 8);
        *reinterpret_cast<u32x4*>(kw + row * RB + (swz_u<HD>(row, ch) << 4)) = v;
      }
    }
    wait_vmcnt<0>();
    __syncthreads();
    // dV^T (key half kh, d tile dt) = asm-owned AGPR block 2 kh + dt, dK^T = 4 + 2 kh + dt
    acc32_zero<0>(); acc32_zero<1>(); acc32_zero<2>(); acc32_zero<3>();
    acc32_zero<4>(); acc32_zero<5>(); acc32_zero<6>(); acc32_zero<7>();
    const __amdgpu_buffer_rsrc_t rdq = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(DQP + (((long long)bh * nkb + kb) * nqt) * kDqChunk), (short)0, nqt * kDqChunk * 4, 0x00020000);
    // dQ^T of query tile tt from dS buffer `buf`: nks 16-key steps (the keys below the tile's end)
    auto dq_steps = [&](f32x16& dq, const char* buf, int s0, int nks) __attribute__((always_inline)) {
#pragma unroll
      for (int h4 = 0; h4 < 2; ++h4) {   // 4 key steps per read batch: K^T and dS^T fragments
        const int sb = s0 + 4 * h4;
        if (sb < nks) {
          s16x4 th[16];
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            th[4 * s] = ds_tr16_off(kst + koff[0], 16 * (sb + s) * RB);
            th[4 * s + 1] = ds_tr16_off(kst + koff[1], 16 * (sb + s) * RB);
            th[4 * s + 2] = ds_tr16_off(buf + doff[0], 16 * (sb + s) * RB);
            th[4 * s + 3] = ds_tr16_off(buf + doff[1], 16 * (sb + s) * RB);
          }
          tr_wait8(th);
#pragma unroll
          for (int s = 0; s < 4; ++s)
            dq = MFMA32(tr_join(th[4 * s], th[4 * s + 1]), tr_join(th[4 * s + 2], th[4 * s + 3]), dq);
        }
      }
    };
    auto dq_store = [&](const f32x16& dq, int tt) __attribute__((always_inline)) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 v = {dq[4 * g], dq[4 * g + 1], dq[4 * g + 2], dq[4 * g + 3]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rdq,
                                               (unsigned)((tt * kDqChunk + wave * 1024 + (g * 64 + l) * 4) * 4), 0, 0);
      }
    };
    auto nks_of = [&](int q0_) { return causal ? min(16, (q0_ + BQ - k0) >> 4) : 16; };

    for (int t = 0; t < nq; ++t) {
      {   // tile t landed (what was issued after its DMA may still fly), dS(t-1) of every wave written
        const int st2 = t >= 3 ? NSTORE : 0, dm1 = t >= 1 && t + 1 < nq ? PWV : 0, st1 = t >= 2 ? NSTORE : 0;
        if (t == 0) wait_vmcnt<0>();
        else wait_vm_rt(st2 + dm1 + st1);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const char* lq = smem + cur * BUF;
      const char* ldo_ = lq + TILE;
      const float* ls = reinterpret_cast<const float*>(lq + 2 * TILE);
      const float* ds = ls + 64;
      int nb = cur + 2;
      if (nb >= NST) nb -= NST;
      cur = (cur + 1 == NST) ? 0 : cur + 1;
      const int q0 = qstart + t * BQ;
      if (t + 2 < nq) dma.issue(qbase, dobase, lsb, dlb, ldq, lddo, T, q0 + 2 * BQ, smem + nb * BUF);
      const char* dsp = dsb + ((t + 1) & 1) * DSB;   // dS of tile t - 1
      char* dsc = dsb + (t & 1) * DSB;               // dS of tile t
      const int nksp = t > 0 ? nks_of(q0 - BQ) : 0;
      f32x16 dq;
#pragma unroll
      for (int i = 0; i < 16; ++i) dq[i] = 0.f;
      const bool act = !causal || kw0 <= q0 + BQ - 1;   // wave-uniform
      if (!act) {
        if (t > 0) {
          dq_steps(dq, dsp, 0, nksp);
          dq_steps(dq, dsp, 8, nksp);
          dq_store(dq, qt0 + t - 1);
        }
        continue;
      }
      const bool need_mask = __builtin_amdgcn_readfirstlane(
          (int)((causal && kw0 + 63 > q0) || (q0 + BQ > T) || (kw0 + 64 > T)));
      const int uq = T - 1 - q0 - 4 * hf;
      int vk[2];
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const int key = kw0 + 32 * kh + r32;
        vk[kh] = key >= T ? 0x7fffffff : (causal ? key - q0 - 4 * hf : -0x7fffffff);
      }
      bf16x8 fa[KS], fb[KS];
      auto load_half = [&](int) __attribute__((always_inline)) {};
      // transposed dO^T / Q^T fragments of query half qt (A of dV^T / dK^T; shared by both key halves)
      s16x4 tho[16];
      auto load_tr = [&](int qt) __attribute__((always_inline)) {
#pragma unroll
        for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
          for (int s1 = 0; s1 < 2; ++s1) {
            const int o = 16 * (2 * qt + s1) * RB;
            tho[4 * (2 * dt + s1)] = ds_tr16_off(ldo_ + toff[dt][0], o);
            tho[4 * (2 * dt + s1) + 1] = ds_tr16_off(ldo_ + toff[dt][1], o);
            tho[4 * (2 * dt + s1) + 2] = ds_tr16_off(lq + toff[dt][0], o);
            tho[4 * (2 * dt + s1) + 3] = ds_tr16_off(lq + toff[dt][1], o);
          }
      };
      f32x16 sc[4], dp[4];      // block j = 2 qt + kh
      bf16x8 pp[4][2], pd[4][2];
      auto sdp = [&](int j) __attribute__((always_inline)) {
        const int qt = j >> 1, kh = j & 1;
        // the row constants are the chains' initial accumulators: S' = S - lse / scale, dP' =
        // dP - delta (rows 32 qt + 8 g + 4 hf + 0..3: four consecutive floats of the stage)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 lv = *reinterpret_cast<const f32x4*>(ls + 32 * qt + 8 * g + 4 * hf);
          const f32x4 dd = *reinterpret_cast<const f32x4*>(ds + 32 * qt + 8 * g + 4 * hf);
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            sc[j][4 * g + jj] = lv[jj];
            dp[j][4 * g + jj] = dd[jj];
          }
        }
        // Q / dO row fragments (A; rows 32 qt + r32): read once per query half (kh 0), issued
        // together with the row constants before the chain
        if (kh == 0) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            fa[ks] = *reinterpret_cast<const bf16x8*>(lq + roff[ks] + 32 * qt * RB);
            fb[ks] = *reinterpret_cast<const bf16x8*>(ldo_ + roff[ks] + 32 * qt * RB);
          }
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          sc[j] = MFMA32(fa[ks], kf[kh][ks], sc[j]);
          dp[j] = MFMA32(fb[ks], vf[kh][ks], dp[j]);
        }
      };
      // p = exp2(c2 S'), masked; dS = p dP'; P / dS packed (B operands of dV^T / dK^T); dS rows
      // to LDS for the next tile's dQ
      auto valu = [&](int j) __attribute__((always_inline)) {
        const int qt = j >> 1, kh = j & 1;
#pragma unroll
        for (int i = 0; i < 16; ++i) sc[j][i] = __builtin_amdgcn_exp2f(vmulf(sc[j][i], c2));
        if (need_mask) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int c = 32 * qt + 8 * (i >> 2) + (i & 3);
            sc[j][i] = (c < vk[kh] || c > uq) ? 0.f : sc[j][i];
          }
        }
#pragma unroll
        for (int s1 = 0; s1 < 2; ++s1)
#pragma unroll
          for (int jj = 0; jj < 8; jj += 2) {
            const int i = 8 * s1 + jj;
            pp[j][s1][jj] = (bf16)sc[j][i];
            pp[j][s1][jj + 1] = (bf16)sc[j][i + 1];
            pd[j][s1][jj] = (bf16)vmulf(sc[j][i], dp[j][i]);
            pd[j][s1][jj + 1] = (bf16)vmulf(sc[j][i + 1], dp[j][i + 1]);
          }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const u32x4 w = __builtin_bit_cast(u32x4, pd[j][g >> 1]);
          const u32x2 v = {w[2 * (g & 1)], w[2 * (g & 1) + 1]};
          ds_write64(dsc + wrow + kh * 32 * RB + ((((4 * qt + g) ^ wsw)) << 4), v);
        }
      };
      auto dvdk = [&](int j) __attribute__((always_inline)) {
        const int kh = j & 1;
#pragma unroll
        for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
          for (int s1 = 0; s1 < 2; ++s1) {
            acc32_mfma_i(2 * kh + dt, tr_join(tho[4 * (2 * dt + s1)], tho[4 * (2 * dt + s1) + 1]), pp[j][s1]);
            acc32_mfma_i(4 + 2 * kh + dt, tr_join(tho[4 * (2 * dt + s1) + 2], tho[4 * (2 * dt + s1) + 3]), pd[j][s1]);
          }
      };
      // G0: S / dP of block 0 (query half 0, key half 0)
      load_half(0);
      sdp(0);
      __builtin_amdgcn_sched_barrier(0);
      // G1: S / dP of block 1, the previous tile's dQ (first half of its keys), softmax-grad of 0
      sdp(1);
      load_half(1);
      if (t > 0) dq_steps(dq, dsp, 0, nksp);
      valu(0);
      load_tr(0);
      __builtin_amdgcn_sched_barrier(0);
      // G2: S / dP of block 2 (query half 1), dV / dK of block 0, softmax-grad of 1
      sdp(2);
      tr_wait8(tho);
      dvdk(0);
      valu(1);
      __builtin_amdgcn_sched_barrier(0);
      // G3: S / dP of block 3, dV / dK of block 1, softmax-grad of 2
      sdp(3);
      dvdk(1);
      valu(2);
      __builtin_amdgcn_sched_barrier(0);
      // G4: the previous tile's dQ (second half), dV / dK of block 2, softmax-grad of 3
      load_tr(1);
      if (t > 0) dq_steps(dq, dsp, 8, nksp);
      tr_wait8(tho);
      dvdk(2);
      valu(3);
      __builtin_amdgcn_sched_barrier(0);
      // G5: dV / dK of block 3; the previous tile's dQ partial out
      dvdk(3);
      if (t > 0) dq_store(dq, qt0 + t - 1);
    }
    // drain: dQ of the last tile (every wave's dS rows written: barrier)
    if (nq > 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __syncthreads();
      const int tl = nq - 1;
      f32x16 dq;
#pragma unroll
      for (int i = 0; i < 16; ++i) dq[i] = 0.f;
      const int nksl = nks_of(qstart + tl * BQ);
      const char* dsl = dsb + (tl & 1) * DSB;
      dq_steps(dq, dsl, 0, nksl);
      dq_steps(dq, dsl, 8, nksl);
      dq_store(dq, qt0 + tl);
    }
    // epilogue per key half: lane = key, registers = d rows 32 dt + 8 g + 4 hf + j.  dK *= scale,
    // inverse RoPE (d pairs with d + HD/2: tile dt with dt + DTN/2, same register)
    acc32_drain();
    f32x16 dkt[2][DTN], dvt[2][DTN];
    dvt[0][0] = acc32_read<0>(); dvt[0][1] = acc32_read<1>(); dvt[1][0] = acc32_read<2>(); dvt[1][1] = acc32_read<3>();
    dkt[0][0] = acc32_read<4>(); dkt[0][1] = acc32_read<5>(); dkt[1][0] = acc32_read<6>(); dkt[1][1] = acc32_read<7>();
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int key = kw0 + 32 * kh + r32;
#pragma unroll
      for (int d = 0; d < DTN; ++d) dkt[kh][d] *= scale;
      if (rpos && key < T) {
        KASSERT(rpos[(long long)b * T + key] >= 0, "rope position at key %d", key);
        const float* tr = rtab + rpos[(long long)b * T + key] * HD;
#pragma unroll
        for (int dt = 0; dt < DTN / 2; ++dt)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 cs = *reinterpret_cast<const f32x4*>(tr + 32 * dt + 8 * g + 4 * hf);
            const f32x4 sn = *reinterpret_cast<const f32x4*>(tr + HD / 2 + 32 * dt + 8 * g + 4 * hf);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float x1 = dkt[kh][dt][4 * g + j], x2 = dkt[kh][dt + DTN / 2][4 * g + j];
              dkt[kh][dt][4 * g + j] = x1 * cs[j] + x2 * sn[j];
              dkt[kh][dt + DTN / 2][4 * g + j] = x2 * cs[j] - x1 * sn[j];
            }
          }
      }
      u32x4 rk[RowStage<HD>::NI], rv[RowStage<HD>::NI];
      RowStage<HD>::put(ep, dkt[kh]);
      RowStage<HD>::get(ep, rk);
      RowStage<HD>::put(ep, dvt[kh]);
      RowStage<HD>::get(ep, rv);
      RowStage<HD>::put_rows(rk, dK + (long long)b * T * lddk + (long long)h * HD, lddk, kw0 + 32 * kh, T);
      RowStage<HD>::put_rows(rv, dV + (long long)b * T * lddv + (long long)h * HD, lddv, kw0 + 32 * kh, T);
    }
    if (BPK) {
      // per-wave column sums over its 64 keys (keys >= T hold zeros): both key halves, then the
      // 32 lanes of each half; the two lane halves hold disjoint d rows
      const long long row = (((long long)h * (BH / H) + b) * nkb + kb) * 4 + wave;
      float wk[DTN * 16], wv[DTN * 16];
#pragma unroll
      for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float a = 0.f, c = 0.f;
#pragma unroll
          for (int kh = 0; kh < 2; ++kh) {
            const bool kv = kw0 + 32 * kh + r32 < T;
            a += kv ? dkt[kh][dt][i] : 0.f;
            c += kv ? dvt[kh][dt][i] : 0.f;
          }
          wk[16 * dt + i] = a;
          wv[16 * dt + i] = c;
        }
      lane32_sums(wk, r32);   // transpose reduction over the 32 lanes of each half
      lane32_sums(wv, r32);
#pragma unroll
      for (int j = 0; j < DTN / 2; ++j) {
        const int rr = r32 * (DTN / 2) + j, i = rr & 15;
        const int d = 32 * (rr >> 4) + 8 * (i >> 2) + 4 * hf + (i & 3);
        BPK[row * HD + d] = wk[j];
        BPV[row * HD + d] = wv[j];
      }
    }
  }
}

// dQ = scale * sum over the key blocks of attn_bwd_fused_k's fp32 partials (in key-block order:
// deterministic), inverse RoPE, bf16 rows; optional per-(b, h, query tile) column sums for the
// q bias gradient.  One workgroup per (query tile of 64, b * H + h); thread t: query t & 63,
// d columns 8 c .. 8 c + 7 and 32 + 8 c .. (c = t >> 6: the RoPE pairs d, d + 32 in one thread).
template <int HD>
__global__ __launch_bounds__(256) void attn_dq_reduce_k(const float* __restrict__ DQP, bf16* __restrict__ dQ, int T,
                                                        int H, long long lddq, float scale, int causal,
                                                        const int64_t* __restrict__ rpos,
                                                        const float* __restrict__ rtab, float* __restrict__ BPQ) {
  static_assert(HD == 64, "dQ reduce: head_dim 64");
  constexpr int KB = 256, BQ = 64;
  const int nkb = (T + KB - 1) / KB, nqt = (T + BQ - 1) / BQ;
  const int qtile = blockIdx.x, bh = blockIdx.y, b = bh / H, h = bh % H;
  const int ql = threadIdx.x & 63, c = threadIdx.x >> 6;
  const int q = qtile * BQ + ql;
  const int kbe = causal ? min(nkb, (qtile * BQ) / KB + 1) : nkb;   // key blocks that saw this tile
  float x[2][8];
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int j = 0; j < 8; ++j) x[dt][j] = 0.f;
  const int w0 = (ql >> 5) * 2, lane = ql & 31;
  for (int kb = 0; kb < kbe; ++kb) {
    const float* base = DQP + (((long long)bh * nkb + kb) * nqt + qtile) * kDqChunk;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(base + (w0 + dt) * 1024 + (c * 64 + 32 * hh + lane) * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) x[dt][4 * hh + j] += v[j];
      }
  }
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int j = 0; j < 8; ++j) x[dt][j] *= scale;
  if (rpos && q < T) {
    const float* tr = rtab + rpos[(long long)b * T + q] * HD;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float cs = tr[8 * c + j], sn = tr[HD / 2 + 8 * c + j];
      const float x1 = x[0][j], x2 = x[1][j];
      x[0][j] = x1 * cs + x2 * sn;
      x[1][j] = x2 * cs - x1 * sn;
    }
  }
  if (q < T) {
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)x[dt][j];
      *reinterpret_cast<bf16x8*>(dQ + ((long long)b * T + q) * lddq + (long long)h * HD + 32 * dt + 8 * c) = v;
    }
  }
  if (BPQ) {
    // column sums over the tile's 64 queries: one wave holds one c (d columns 8 c.., 32 + 8 c..)
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a = q < T ? x[dt][j] : 0.f;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) a += __shfl_xor(a, o, 64);
        if (ql == 0) BPQ[((long long)h * (gridDim.y / H) + b) * nqt * HD + (long long)qtile * HD + 32 * dt + 8 * c + j] = a;
      }
  }
}

}  // namespace dpfs

using namespace dpfs;

// Fused backward (impl 6, head_dim 64): attn_bwd_delta_k -> attn_bwd_fused_k -> attn_dq_reduce_k
// (+ the bias-gradient reduction).  dqp: dpfs_attn_fused_ws floats of fp32 dQ partials;
// delta: [2][B, H, T] fp32 (-delta | -lse/scale); bws: dpfs_attn_fused_bias_ws floats when
// dbias is requested.
// ================================= bwd: dK, dV, 64 keys per wave (one wave per SIMD) ==
// attn_bwd_dkdv3_k with each wave owning 64 keys (two 32-key halves kh) instead of 32: every Q /
// dO fragment read from LDS (rows for S / dP, transposed for dV^T / dK^T) feeds twice the MFMAs,
// which halves the LDS traffic per MFMA (the v3 kernel moves as many LDS bytes per CU as its
// MFMAs take cycles), and a workgroup's prologue (K / V to registers, the first two tiles) is
// paid once per 256 keys.  The accumulators (dK^T / dV^T of 64 keys: 128 floats per lane) and
// the K / V operands no longer leave room for a second wave per SIMD: a workgroup = 4 waves x 64
// keys per CU, and the VALU softmax work of one key half overlaps the other half's MFMAs inside
// the wave.  head_dim 64; same operands, row constants, ring and epilogue as v3.  dV^T / dK^T
// of key half kh, d tile dt are the asm-owned AGPR blocks 2 kh + dt / 4 + 2 kh + dt
// (attn_acc.inc), so the compiler's 256 VGPRs hold everything else.
template <int HD>
__global__ __launch_bounds__(256, 1) void attn_bwd_dkdv4_k(
    const bf16* __restrict__ Q, const bf16* __restrict__ K, const bf16* __restrict__ V, const bf16* __restrict__ dO,
    const float* __restrict__ LSN, const float* __restrict__ NDEL, bf16* __restrict__ dK, bf16* __restrict__ dV,
    int T, int H, int BH, long long ldq, long long ldk, long long ldv, long long lddo, long long lddk,
    long long lddv, float scale, int causal, const int64_t* __restrict__ rpos, const float* __restrict__ rtab,
    float* __restrict__ BPK, float* __restrict__ BPV, int prefetch = 1) {
  static_assert(HD == 64, "dK/dV v4: head_dim 64");
  constexpr int BK = 256, BQ = 64, KS = HD / 16, DTN = HD / 32, RB = HD * 2;
  constexpr int TILE = BQ * RB, BUF = 2 * TILE + 1024, NST = 3;
  constexpr int PWV = QdoDma3<HD>::PW + 1;
  __shared__ __attribute__((aligned(1024))) char smem[NST * BUF + 4 * RowStage<HD>::BYTES];
  const int nkb = (T + BK - 1) / BK;
  const int NP = (nkb + 1) / 2;
  const int nkb3 = (T + 127) / 128;   // the bias partials' 32-key rows (v3's layout)
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
  const int kb1 = nkb - 1 - p;
  const int qstart1 = causal ? ((kb1 * BK) / BQ) * BQ : 0;
  const int nq1 = (T - qstart1 + BQ - 1) / BQ;
  const int kw1 = kb1 * BK + 64 * wave;
  const int nq0 = (T - (causal ? ((p * BK) / BQ) * BQ : 0) + BQ - 1) / BQ;
  const bool pre = (prefetch & 1) && kb1 != p && nq1 > 0 && nq0 >= 2;  // (uniform)
  bf16x8 kf[2][KS], vf[2][KS];
  auto load_kv = [&](int kw_) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int kk_ = kw_ + 32 * kh + r32;
        bf16x8 a_ = {}, c_ = {};
        if (kk_ < T) {
          a_ = *reinterpret_cast<const bf16x8*>(K + ((long long)b * T + kk_) * ldk + (long long)h * HD + 16 * ks + 8 * hf);
          c_ = *reinterpret_cast<const bf16x8*>(V + ((long long)b * T + kk_) * ldv + (long long)h * HD + 16 * ks + 8 * hf);
        }
        kf[kh][ks] = a_;
        vf[kh][ks] = c_;
      }
  };
  int cur = 0;
  for (int sub = 0; sub < 2; ++sub) {
    const int kb = sub == 0 ? p : nkb - 1 - p;
    if (sub == 1 && kb == p) break;
    if (sub == 1) __syncthreads();
    const int k0 = kb * BK, kw0 = k0 + 64 * wave;
    const int qstart = causal ? (k0 / BQ) * BQ : 0;
    const int nq = (T - qstart + BQ - 1) / BQ;
    const bool fetched = sub == 1 && pre;
    if (!fetched) {
      const int c1 = cur + 1 == NST ? 0 : cur + 1;
      if (nq > 0) dma.issue(qbase, dobase, lsb, dlb, ldq, lddo, T, qstart, smem + cur * BUF);
      if (nq > 1) dma.issue(qbase, dobase, lsb, dlb, ldq, lddo, T, qstart + BQ, smem + c1 * BUF);
      load_kv(kw0);
    }
    wait_vmcnt<0>();
    // K pre-scaled by scale log2(e) (the dQ kernel's LSN = -lse log2(e) convention, as v3's KSC)
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) kf[kh][ks][j] = (bf16)((float)kf[kh][ks][j] * c2);
    acc32_zero<0>(); acc32_zero<1>(); acc32_zero<2>(); acc32_zero<3>();
    acc32_zero<4>(); acc32_zero<5>(); acc32_zero<6>(); acc32_zero<7>();
    const bool ahead = sub == 0 && pre;
    for (int t = 0; t < nq; ++t) {
      if (t + 1 < nq || ahead) wait_vmcnt<PWV>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      const char* lq = smem + cur * BUF;
      const char* ldo_ = lq + TILE;
      const float* ls = reinterpret_cast<const float*>(lq + 2 * TILE);
      const float* ds = ls + 64;
      int nb = cur + 2;
      if (nb >= NST) nb -= NST;
      cur = (cur + 1 == NST) ? 0 : cur + 1;
      const int q0 = qstart + t * BQ;
      if (t + 2 < nq) dma.issue(qbase, dobase, lsb, dlb, ldq, lddo, T, q0 + 2 * BQ, smem + nb * BUF);
      else if (ahead && t + 2 - nq < nq1)
        dma.issue(qbase, dobase, lsb, dlb, ldq, lddo, T, qstart1 + (t + 2 - nq) * BQ, smem + nb * BUF);
      if (causal && q0 + BQ - 1 < kw0) {   // wave-uniform: every query of the tile < every key
        if (ahead && t == nq - 1) load_kv(kw1);
        continue;
      }
      // S / dP for both query halves qt and key halves kh (rows = queries, lane = key), the
      // row constants as initial accumulators (as v3)
      f32x16 sc[2][2], dp[2][2];
      bf16x8 fa[KS], fb[KS];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 lv = *reinterpret_cast<const f32x4*>(ls + 8 * g + 4 * hf);
        const f32x4 dd = *reinterpret_cast<const f32x4*>(ds + 8 * g + 4 * hf);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sc[0][0][4 * g + j] = lv[j];
          dp[0][0][4 * g + j] = dd[j];
        }
      }
      sc[0][1] = sc[0][0];
      dp[0][1] = dp[0][0];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        fa[ks] = *reinterpret_cast<const bf16x8*>(lq + roff[ks]);
        fb[ks] = *reinterpret_cast<const bf16x8*>(ldo_ + roff[ks]);
      }
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 ga[KS], gb[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        sc[0][0] = MFMA32(fa[ks], kf[0][ks], sc[0][0]);
        sc[0][1] = MFMA32(fa[ks], kf[1][ks], sc[0][1]);
        dp[0][0] = MFMA32(fb[ks], vf[0][ks], dp[0][0]);
        dp[0][1] = MFMA32(fb[ks], vf[1][ks], dp[0][1]);
        ga[ks] = *reinterpret_cast<const bf16x8*>(lq + roff[ks] + 32 * RB);
        gb[ks] = *reinterpret_cast<const bf16x8*>(ldo_ + roff[ks] + 32 * RB);
        if (ks < 2) {
#pragma unroll
          for (int g = 2 * ks; g < 2 * ks + 2; ++g) {
            const f32x4 lv = *reinterpret_cast<const f32x4*>(ls + 32 + 8 * g + 4 * hf);
            const f32x4 dd = *reinterpret_cast<const f32x4*>(ds + 32 + 8 * g + 4 * hf);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              sc[1][0][4 * g + j] = lv[j];
              dp[1][0][4 * g + j] = dd[j];
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      sc[1][1] = sc[1][0];
      dp[1][1] = dp[1][0];
      // query half 1's MFMAs, half 0's exponentials under them (8 per k-step and key half)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        sc[1][0] = MFMA32(ga[ks], kf[0][ks], sc[1][0]);
        sc[1][1] = MFMA32(ga[ks], kf[1][ks], sc[1][1]);
        dp[1][0] = MFMA32(gb[ks], vf[0][ks], dp[1][0]);
        dp[1][1] = MFMA32(gb[ks], vf[1][ks], dp[1][1]);
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int i = (16 / KS) * ks; i < (16 / KS) * (ks + 1); ++i)
            sc[0][kh][i] = __builtin_amdgcn_exp2f(sc[0][kh][i]);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (ahead && t == nq - 1) load_kv(kw1);
      // dO^T fragments (A of dV^T), shared by both key halves
      constexpr int NH = 2 * DTN * 4;
      s16x4 th[NH];
#pragma unroll
      for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          th[2 * (dt * 4 + s4)] = ds_tr16_off(ldo_ + toff[dt][0], 16 * s4 * RB);
          th[2 * (dt * 4 + s4) + 1] = ds_tr16_off(ldo_ + toff[dt][1], 16 * s4 * RB);
        }
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int i = 0; i < 16; ++i) sc[1][kh][i] = __builtin_amdgcn_exp2f(sc[1][kh][i]);
      const bool need_mask = __builtin_amdgcn_readfirstlane(
          (int)((causal && kw0 + 63 > q0) || (q0 + BQ > T) || (kw0 + 64 > T)));
      if (need_mask) {
        const int uq = T - 1 - q0 - 4 * hf;
#pragma unroll
        for (int kh = 0; kh < 2; ++kh) {
          const int key = kw0 + 32 * kh + r32;
          const int vk = key >= T ? 0x7fffffff : (causal ? key - q0 - 4 * hf : -0x7fffffff);
#pragma unroll
          for (int qt = 0; qt < 2; ++qt)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int c = 32 * qt + 8 * (i >> 2) + (i & 3);
              sc[qt][kh][i] = (c < vk || c > uq) ? 0.f : sc[qt][kh][i];
            }
        }
      }
      // P and dS = p (dP - delta) packed to bf16: operand pp[kh][s4] / pd[kh][s4] holds the
      // 16-query k-step s4 = 2 qt + s1
      bf16x8 pp[2][4], pd[2][4];
#pragma unroll
      for (int kh = 0; kh < 2; ++kh)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int s1 = 0; s1 < 2; ++s1)
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
              const int i = 8 * s1 + j;
              pp[kh][2 * qt + s1][j] = (bf16)sc[qt][kh][i];
              pp[kh][2 * qt + s1][j + 1] = (bf16)sc[qt][kh][i + 1];
              pd[kh][2 * qt + s1][j] = (bf16)vmulf(sc[qt][kh][i], dp[qt][kh][i]);
              pd[kh][2 * qt + s1][j + 1] = (bf16)vmulf(sc[qt][kh][i + 1], dp[qt][kh][i + 1]);
            }
      tr_wait8(*reinterpret_cast<s16x4(*)[16]>(&th[0]));
#pragma unroll
      for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const bf16x8 a = tr_join(th[2 * (dt * 4 + s4)], th[2 * (dt * 4 + s4) + 1]);
          acc32_mfma_i(dt, a, pp[0][s4]);
          acc32_mfma_i(2 + dt, a, pp[1][s4]);
        }
      __builtin_amdgcn_sched_barrier(0);
      // Q^T fragments (A of dK^T), read after the dV^T MFMAs are issued
#pragma unroll
      for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          th[2 * (dt * 4 + s4)] = ds_tr16_off(lq + toff[dt][0], 16 * s4 * RB);
          th[2 * (dt * 4 + s4) + 1] = ds_tr16_off(lq + toff[dt][1], 16 * s4 * RB);
        }
      tr_wait8(*reinterpret_cast<s16x4(*)[16]>(&th[0]));
#pragma unroll
      for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const bf16x8 a = tr_join(th[2 * (dt * 4 + s4)], th[2 * (dt * 4 + s4) + 1]);
          acc32_mfma_i(4 + dt, a, pd[0][s4]);
          acc32_mfma_i(6 + dt, a, pd[1][s4]);
        }
    }
    // epilogue per key half: dK *= scale, inverse RoPE, whole-row stores, bias partials
    acc32_drain();
    f32x16 dkt[2][DTN], dvt[2][DTN];
    dvt[0][0] = acc32_read<0>(); dvt[0][1] = acc32_read<1>(); dvt[1][0] = acc32_read<2>(); dvt[1][1] = acc32_read<3>();
    dkt[0][0] = acc32_read<4>(); dkt[0][1] = acc32_read<5>(); dkt[1][0] = acc32_read<6>(); dkt[1][1] = acc32_read<7>();
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      const int kwh = kw0 + 32 * kh, key = kwh + r32;
#pragma unroll
      for (int d = 0; d < DTN; ++d) dkt[kh][d] *= scale;
      if (rpos && key < T) {
        KASSERT(rpos[(long long)b * T + key] >= 0, "rope position at key %d", key);
        const float* tr = rtab + rpos[(long long)b * T + key] * HD;
#pragma unroll
        for (int dt = 0; dt < DTN / 2; ++dt)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 cs = *reinterpret_cast<const f32x4*>(tr + 32 * dt + 8 * g + 4 * hf);
            const f32x4 sn = *reinterpret_cast<const f32x4*>(tr + HD / 2 + 32 * dt + 8 * g + 4 * hf);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float x1 = dkt[kh][dt][4 * g + j], x2 = dkt[kh][dt + DTN / 2][4 * g + j];
              dkt[kh][dt][4 * g + j] = x1 * cs[j] + x2 * sn[j];
              dkt[kh][dt + DTN / 2][4 * g + j] = x2 * cs[j] - x1 * sn[j];
            }
          }
      }
      {
        u32x4 rk[RowStage<HD>::NI], rv[RowStage<HD>::NI];
        RowStage<HD>::put(ep, dkt[kh]);
        RowStage<HD>::get(ep, rk);
        RowStage<HD>::put(ep, dvt[kh]);
        RowStage<HD>::get(ep, rv);
        RowStage<HD>::put_rows(rk, dK + (long long)b * T * lddk + (long long)h * HD, lddk, kwh, T);
        RowStage<HD>::put_rows(rv, dV + (long long)b * T * lddv + (long long)h * HD, lddv, kwh, T);
      }
      const int u = kwh >> 5;   // the 32-key row of the bias partials (v3 layout)
      if (BPK && u < 4 * nkb3) {
        const long long row = (((long long)h * (BH / H) + b) * nkb3 + (u >> 2)) * 4 + (u & 3);
        float wk[DTN * 16], wv[DTN * 16];   // the v3 kernel's transpose reduction (lane32_sums)
#pragma unroll
        for (int dt = 0; dt < DTN; ++dt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            wk[16 * dt + i] = key < T ? dkt[kh][dt][i] : 0.f;
            wv[16 * dt + i] = key < T ? dvt[kh][dt][i] : 0.f;
          }
        lane32_sums(wk, r32);
        lane32_sums(wv, r32);
#pragma unroll
        for (int j = 0; j < DTN / 2; ++j) {
          const int rr = r32 * (DTN / 2) + j, i = rr & 15;
          const int d = 32 * (rr >> 4) + 8 * (i >> 2) + 4 * hf + (i & 3);
          BPK[row * HD + d] = wk[j];
          BPV[row * HD + d] = wv[j];
        }
      }
    }
  }
}


extern "C" void dpfs_attn_bwd_dkdv4(int items, const void* q, const void* k, const void* v, const void* dout,
                                    const float* lsn, const float* ndel, void* dk, void* dv, int T, int H, int BH,
                                    long long ldq, long long ldk, long long ldv, long long lddo, long long lddk,
                                    long long lddv, float scale, int causal, const int64_t* rope_pos,
                                    const float* rope_tab, float* pk, float* pv, int prefetch, hipStream_t s) {
  attn_bwd_dkdv4_k<64><<<items, 256, 0, s>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (const bf16*)dout, lsn,
                                              ndel, (bf16*)dk, (bf16*)dv, T, H, BH, ldq, ldk, ldv, lddo, lddk, lddv,
                                              scale, causal, rope_pos, rope_tab, pk, pv, prefetch);
}

extern "C" long long dpfs_attn_fused_ws(int B, int T, int H, int hd) {
  if (hd != 64) return -1;
  const long long nkb = (T + 255) / 256, nqt = (T + 63) / 64;
  return (long long)B * H * nkb * nqt * kDqChunk;
}
extern "C" long long dpfs_attn_fused_bias_ws(int B, int T, int H, int hd) {
  const long long nkb = (T + 255) / 256, nqt = (T + 63) / 64;
  return (long long)H * B * (nqt + 2 * nkb * 4) * hd;
}
extern "C" int dpfs_attn_bwd_fused(const void* dout, const void* q, const void* k, const void* v, const void* o,
                                   const float* lse, float* delta, float* dqp, void* dq, void* dk, void* dv, int B,
                                   int T, int H, int hd, long long lddo, long long ldq, long long ldk, long long ldv,
                                   long long ldo, long long lddq, long long lddk, long long lddv, float scale,
                                   int causal, const int64_t* rope_pos, const float* rope_tab, hipStream_t s,
                                   float* dbias, float* bws) {
  if (hd != 64) return -1;
  const bool bias = dbias != nullptr && bws != nullptr;
  const long long rows = (long long)B * T * H;
  const int nkb = (T + 255) / 256, nqt = (T + 63) / 64;
  float* ndel = delta;
  float* lsn = delta + (long long)B * H * T;
  attn_bwd_delta_k<64><<<(unsigned)((rows * 8 + 255) / 256), 256, 0, s>>>(
      (const bf16*)dout, (const bf16*)o, lse, ndel, lsn, T, H, rows, lddo, ldo, 1.f / scale);
  float* pq = bias ? bws : nullptr;
  float* pk = bias ? bws + (long long)H * B * nqt * hd : nullptr;
  float* pv = bias ? pk + (long long)H * B * nkb * 4 * hd : nullptr;
  const int items = (B * H + 7) / 8 * 8 * ((nkb + 1) / 2);
  attn_bwd_fused_k<64><<<items, 256, 0, s>>>((const bf16*)q, (const bf16*)k, (const bf16*)v, (const bf16*)dout, lsn,
                                             ndel, (bf16*)dk, (bf16*)dv, dqp, T, H, B * H, ldq, ldk, ldv, lddo, lddk,
                                             lddv, scale, causal, rope_pos, rope_tab, pk, pv);
  attn_dq_reduce_k<64><<<dim3(nqt, B * H), 256, 0, s>>>(dqp, (bf16*)dq, T, H, lddq, scale, causal, rope_pos, rope_tab,
                                                        pq);
  if (bias) {
    attn_bias_grad_k<64><<<3 * H * 4, 1024, 0, s>>>(pq, pk, pv, dbias, H, B * nqt, B * nkb * 4);
    return 1;
  }
  return 0;
}
