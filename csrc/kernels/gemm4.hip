// bf16 MFMA GEMM v4 for gfx950 (MI355X): one wave per SIMD, 128 x 128 outputs per wave.
//
//   C[m][n] = sum_k A(m,k) B(k,n), fp32 accumulation in the accumulator (AGPR) file.
//   Layouts as gemm.hip: NT forward (F.linear, reference models/layers.py:49,93), NN dgrad,
//   TN wgrad (fp32 split-K slabs).
//
// Why a new main loop (the v3 kernel in gemm.hip runs 8 waves, 2 per SIMD, 128 x 64 each):
//  * 128 x 128 per wave halves the LDS bytes read per MFMA (16 ds_read_b128 per 64
//    v_mfma_f32_16x16x32_bf16 = 0.25, v3 0.375) and one wave per SIMD leaves each SIMD's
//    matrix pipe to one instruction stream.  The 256 fp32 accumulators per lane are
//    asm-owned AGPRs a[0:255] (gemm4_acc.inc, generated): hipcc never moves or spills them,
//    and fragments, addresses and the epilogue get the 256 arch VGPRs.
//  * The K loop walks 32-deep steps through a 4-slot LDS ring (32 KiB per slot: A and B
//    256 x 32 bf16 each).  Step s multiplies fragments already in registers, reads the next
//    step's fragments in its first half (one step of register prefetch: no LDS latency at a
//    step boundary) and issues the LDS-DMA of step s + 3 in its second half (two full steps
//    for each DMA to land).  One barrier per step; counted `s_waitcnt vmcnt` (never 0 in
//    the loop).  Fragment reads and DMA pieces sit between MFMA pairs in a fixed order
//    (sched_barrier), the DMA offsets are per-item lane constants plus one uniform add.
//  * Persistent: one 256-thread workgroup per CU walks (split, tile) items in grouped,
//    XCD-contiguous order; the DMA stream continues across item boundaries, so the next
//    item's first three steps are in flight while an item's epilogue runs.  Past the last
//    item the producer issues out-of-range DMAs (zeros into dead slots) so every wait count
//    stays static.
//  * Epilogue: the wave's 128 bias values arrive in its own LDS area by LDS-DMA issued at the
//    item's last step (a counted vmcnt, no ring drain); bias (+ RoPE for the QKV projection,
//    head_dim 64 or 128: the rotation partner of column d is d + hd/2, the same lane's tile
//    j + hd/32) in fp32, bf16; v_permlane16_swap pairs two 16-column tiles so each lane
//    writes 8 consecutive columns with one 16-byte buffer store.  Out-of-range rows /
//    columns get an offset past the descriptor (dropped by hardware).
//  * LDS images: K-contiguous operands [256 rows][64 B] with the 16-byte chunk of row r at
//    slot c ^ h(r), h(r) = (-(r >> 2)) & 3: every ds_read_b128 lane group covers the 16 bank
//    slots exactly once.  MN-contiguous operands [32 k][256] as gemm.hip (read with the
//    ds_read_b64_tr_b16 hardware transpose, through inline asm: see ds_tr16).  The swizzle
//    is applied on the DMA SOURCE address (LDS-DMA writes lane-linear 1 KiB pieces).
#include "common.h"

#include <algorithm>
#include <type_traits>

namespace dpfs {
namespace g4 {

#include "gemm4_acc.inc"

constexpr int SLOT = 32768;          // one ring slot: A (16 KiB) + B (16 KiB)
constexpr int RING = 4 * SLOT;       // 128 KiB
constexpr int BIAS_LDS = 4 * 512;    // per wave: its 128 fp32 bias values
constexpr int LDS_TOTAL = RING + BIAS_LDS;

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

__device__ __forceinline__ int kh(int r) { return (4 - ((r >> 2) & 3)) & 3; }
__device__ __forceinline__ int mnh(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

struct Rope {
  const int64_t* pos;
  const float* tab;   // [maxlen][hd] = [cos(0..hd/2) | sin(0..hd/2)]
  int cols;           // rotate output columns < cols (q and k heads)
  int hd;             // 64 or 128
};

// SwiGLU in the gate|up projection's epilogue (reference models/model.py:94-95): the packed
// [gate | up] weight (natural layout) is read with its rows interleaved in 64-row blocks
// (reference.gu_perm: output columns [128 b, 128 b + 64) = gate rows [64 b, 64 b + 64), the
// next 64 = the matching up rows; the mapping is applied to the DMA pieces' row offsets and the
// bias offsets, no copy), so a wave's 128 columns hold 64 gate / up pairs in the same lane
// (tiles j and j + 4).  Besides the (interleaved) gate|up output, h[:, 64 b + c] =
// silu(gate) * up of the bf16-rounded values -- the swiglu_fwd_k arithmetic, bit for bit.
__device__ __forceinline__ int gu_nat(int c, int F) {   // interleaved column -> natural row
  const int b = c >> 7, r = c & 127;
  return r < 64 ? (b << 6) + r : F + (b << 6) + r - 64;
}
struct SwiOut {
  bf16* h;
  int ldh;
  unsigned h_bytes;
};

// SwiGLU backward in the down projection's data-gradient epilogue (NN layout; reference
// models/model.py:94-95, differentiated): the GEMM's C = ds = dy W_down (the gradient wrt
// h = silu(gate) * up) never reaches memory.  Per element the epilogue rounds ds to bf16 (the
// value the separate pass would have read), loads gate / up from the forward's gu (interleaved
// 64-column blocks when `perm`, else natural [gate | up]) and writes
//   dgate = ds * up * s * (1 + gate * (1 - s)),  dup = ds * gate * s,  s = sigmoid(gate)
// to dgu in the natural [gate | up] layout -- the swiglu_bwd_colsum_k arithmetic.  The gate|up
// bias gradient (column sums of dgu) comes out as fp32 partials, one row per wave's 128 rows:
// part[(m0 + 128 wm) / 128][2F], summed over the lane's 8 row blocks in registers and over the
// 16 lanes of a DPP row (fixed order, deterministic); colsum_rows reduces the partial rows.
struct SwiBwd {
  const bf16* gu;
  bf16* dgu;
  float* part;
  int ldgu, lddgu, perm;
  unsigned gu_bytes, dgu_bytes, part_bytes;
};

struct Dual {
  const bf16* A2;
  const bf16* B2;
  int k_switch, lda2, ldb2;
  unsigned a2_bytes, b2_bytes;
};

// Fragment of the 16x16x32 MFMA operand: lane l holds X[rb + (l&15)][8(l>>4) + e], e < 8.
__device__ __forceinline__ bf16x8 frag_k(const char* half, int rb, int l) {
  const int row = rb + (l & 15);
  const int c = l >> 4;
  return *reinterpret_cast<const bf16x8*>(half + row * 64 + ((c ^ kh(row)) << 4));
}

// MN-major fragment halves through inline asm: hipcc puts `s_waitcnt vmcnt(0)` in front of
// the ds_read_b64_tr_b16 builtin whenever an LDS-DMA is in flight (it cannot tell the DMA's
// LDS destination from the read's), which would drain the ring at every read.  The asm form
// is invisible to that bookkeeping; Opnd::pin retires the reads with one `s_waitcnt
// lgkmcnt(0)` naming every destination "+v" before any use (guide §5.7 item 1, form (ii)).
__device__ __forceinline__ s16x4 ds_tr16(const char* p) {
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"((unsigned)(size_t)((__attribute__((address_space(3))) const char*)p)));
  return r;
}

// BN: the operand tile's MN extent (256, or 192 for the B operand of a 256 x 192 tile).  An
// MN-major image keeps BN * 2 bytes per k row; at BN = 192 the chunk swizzle stays inside
// each aligned group of 8 chunks, so a swizzled chunk index never leaves the row's 24.
template <int BN>
__device__ __forceinline__ int mn_swz(int k) {
  return BN == 256 ? mnh(k) << 1 : (mnh(k) & 3) << 1;
}

template <bool KMAJ, int BN = 256>
struct Opnd;
template <int BN>
struct Opnd<true, BN> {
  bf16x8 v[8];
  __device__ __forceinline__ void load(int i, const char* half, int rb, int l) { v[i] = frag_k(half, rb, l); }
  __device__ __forceinline__ bf16x8 get(int i) const { return v[i]; }
  __device__ __forceinline__ void pin() {}
};
template <int BN>
struct Opnd<false, BN> {
  s16x4 lo[8], hi[8];
  __device__ __forceinline__ void load(int i, const char* half, int rb, int l) {
    const int ii = l & 15, q = ii >> 2, p = ii & 3;
    const int chunk = (rb + 4 * p) >> 3;
    const int k_lo = 8 * (l >> 4) + q;
    const int k_hi = k_lo + 4;
    lo[i] = ds_tr16(half + k_lo * (2 * BN) + ((chunk ^ mn_swz<BN>(k_lo)) << 4) + (p & 1) * 8);
    hi[i] = ds_tr16(half + k_hi * (2 * BN) + ((chunk ^ mn_swz<BN>(k_hi)) << 4) + (p & 1) * 8);
  }
  __device__ __forceinline__ bf16x8 get(int i) const {
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[i][0], lo[i][1], lo[i][2], lo[i][3], hi[i][0], hi[i][1], hi[i][2], hi[i][3]};
    return __builtin_bit_cast(bf16x8, v);
  }
  __device__ __forceinline__ void pin() {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(lo[0]), "+v"(lo[1]), "+v"(lo[2]), "+v"(lo[3]), "+v"(lo[4]), "+v"(lo[5]), "+v"(lo[6]),
                   "+v"(lo[7]));
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(hi[0]), "+v"(hi[1]), "+v"(hi[2]), "+v"(hi[3]), "+v"(hi[4]), "+v"(hi[5]), "+v"(hi[6]),
                   "+v"(hi[7]));
  }
};

// 32x32x16 operand of an MN-major image (the M32 main loop): fragment f = 2 nb + kk covers the
// wave's 32-column block nb (of 4) and k-half kk: lane l holds X[k = 16 kk + 8 (l >> 5) + j]
// [col 32 nb + (l & 31)], j < 8, from two ds_read_b64_tr_b16 (rows k, k + 4 of its 16-lane
// group's 4 x 16 block: group g takes columns 16 (g & 1) .. + 15 and k half g >> 1).  The
// image's 16-byte chunk c of k row r sits at c ^ ((r & 3) << 2): the four rows of a 32-lane
// half's two blocks (64 contiguous bytes each) land on four disjoint 4-chunk bank groups.
__device__ __forceinline__ int m32_swz(int k) { return (k & 3) << 2; }
// transposed read at a compile-time byte offset from p (the ds instruction's offset field)
template <int OFF>
__device__ __forceinline__ s16x4 ds_tr16_at(const char* p) {
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2"
               : "=v"(r)
               : "v"((unsigned)(size_t)((__attribute__((address_space(3))) const char*)p)), "n"(OFF));
  return r;
}
// Lane offset of fragment block nb (k-half 0, rows k, the lo read) in a half-slot: the other
// three reads of the block are +2048 (rows k + 4), +8192 (k-half 1) and +10240, so a step
// needs one address add per block (the swizzle depends on k & 3 only).
__device__ __forceinline__ unsigned m32_off(int cb, int nb, int l) {
  const int ii = l & 15, q = ii >> 2, p = ii & 3, g = l >> 4;
  const int col = cb + 32 * nb + 16 * (g & 1) + 4 * p;
  const int k = 8 * (g >> 1) + q;
  return (unsigned)(k * 512 + (((col >> 3) ^ m32_swz(k)) << 4) + (p & 1) * 8);
}
struct Opnd32 {
  s16x4 lo[8], hi[8];
  // fragments 2 nb (k-half 0) and 2 nb + 1 (k-half 1) from base = half-slot + m32_off(nb)
  __device__ __forceinline__ void load_nb(int nb, const char* base) {
    lo[2 * nb] = ds_tr16_at<0>(base);
    hi[2 * nb] = ds_tr16_at<2048>(base);
    lo[2 * nb + 1] = ds_tr16_at<8192>(base);
    hi[2 * nb + 1] = ds_tr16_at<10240>(base);
  }
  __device__ __forceinline__ bf16x8 get(int f) const {
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[f][0], lo[f][1], lo[f][2], lo[f][3], hi[f][0], hi[f][1], hi[f][2], hi[f][3]};
    return __builtin_bit_cast(bf16x8, v);
  }
  __device__ __forceinline__ void pin() {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(lo[0]), "+v"(lo[1]), "+v"(lo[2]), "+v"(lo[3]), "+v"(lo[4]), "+v"(lo[5]), "+v"(lo[6]),
                   "+v"(lo[7]));
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(hi[0]), "+v"(hi[1]), "+v"(hi[2]), "+v"(hi[3]), "+v"(hi[4]), "+v"(hi[5]), "+v"(hi[6]),
                   "+v"(hi[7]));
  }
};

// 32x32x16 operand of a K-contiguous image ([256 rows][64 B], chunk c of row r at slot
// c ^ kh(r)): fragment f = 2 nb + kk holds X[row 32 nb + (l & 31)][k = 16 kk + 8 (l >> 5) + j],
// j < 8, one ds_read_b128.  kh(row) depends on row & 15 only, so block nb is +2048 bytes (an
// immediate) from the lane's k-half offset k32_off(kk); each 16-lane group reads 16 rows of one
// chunk, which the swizzle spreads over all 16 bank slots (as the 16x16x32 fragments).
__device__ __forceinline__ unsigned k32_off(int rb, int kk, int l) {
  const int r = l & 31;
  return (unsigned)((rb + r) * 64 + (((2 * kk + (l >> 5)) ^ kh(r)) << 4));
}
struct Opnd32K {
  bf16x8 v[8];
  // fragments 2 nb and 2 nb + 1 from p0 / p1 = half-slot + k32_off(rb, 0 / 1)
  __device__ __forceinline__ void load_nb(int nb, const char* p0, const char* p1) {
    v[2 * nb] = *reinterpret_cast<const bf16x8*>(p0 + 2048 * nb);
    v[2 * nb + 1] = *reinterpret_cast<const bf16x8*>(p1 + 2048 * nb);
  }
  __device__ __forceinline__ bf16x8 get(int f) const { return v[f]; }
  __device__ __forceinline__ void pin() {}
};

template <bool AK, bool BKM, int BN, bool M32 = false>
struct Frags {
  Opnd<AK> a;
  Opnd<BKM, BN> b;
};
template <int BN>
struct Frags<false, false, BN, true> {
  Opnd32 a, b;
};
template <int BN>
struct Frags<true, false, BN, true> {
  Opnd32K a;
  Opnd32 b;
};
template <int BN>
struct Frags<true, true, BN, true> {
  Opnd32K a, b;
};

template <bool AK, bool BKM, int BN, bool M32 = false>
__device__ __forceinline__ void read_frags(Frags<AK, BKM, BN, M32>& f, const char* slot, int wm, int wn, int l) {
  if constexpr (M32) {
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      if constexpr (AK) f.a.load_nb(nb, slot + k32_off(wm * 128, 0, l), slot + k32_off(wm * 128, 1, l));
      else f.a.load_nb(nb, slot + m32_off(wm * 128, nb, l));
    }
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      if constexpr (BKM) f.b.load_nb(nb, slot + 16384 + k32_off(wn * 128, 0, l), slot + 16384 + k32_off(wn * 128, 1, l));
      else f.b.load_nb(nb, slot + 16384 + m32_off(wn * 128, nb, l));
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) f.a.load(i, slot, wm * 128 + 16 * i, l);
#pragma unroll
    for (int j = 0; j < BN / 32; ++j) f.b.load(j, slot + 16384, wn * (BN / 2) + 16 * j, l);
  }
}

// Work item -> tile origin and K range (grouped order as gemm.hip's gemmp_k).
struct Item {
  int m0, n0, kb, ke, split, sel, g;
  int role;   // SK: 0 = whole tile, 1 = first K half (fp32 partial out), 2 = second K half (+ partial)
};

// Stream-K bf16 GEMM (gemm4_k's SK) for the shapes whose 256 x 256 tiles come out at 1.5 per CU
// (N = 768 at 32k rows: 384 tiles on 256 CUs; the 256 x 192 split of the same output runs two
// rounds of narrower, less MFMA-dense tiles).  With G workgroups and E = G / 2 extra tiles,
// workgroup c runs two items: c < E: the first K half of extra tile G + c, then whole tile c;
// c >= E: whole tile c, then the second K half of extra tile G + c - E.  The first half goes
// out as an fp32 partial (write-through, system-coherent stores, drained) with a per-wave
// flag; the second half's epilogue waits for that flag (bounded: s_memrealtime, error word on
// timeout, never a hang) and adds the partial before bias / bf16 / stores.  The producer runs
// its half FIRST and the consumer LAST, so the wait is normally already satisfied.
struct SkArgs {
  float* part;        // [E][4 waves][64 x 64 lanes x 4] fp32, lane-linear per wave
  unsigned* flags;    // [E][4 waves], zeroed before the launch; 1 = partial written
  unsigned* err;      // host-mapped, sticky: set to 1 when a wait timed out (dpfs_gemm4_sk_error)
  int extra;          // E
  int starve;         // test hook: producers never raise their flags (every wait times out)
};
constexpr int kAuxSys = 1 | 16;   // sc0 | sc1: write-through stores, L2-bypassing loads

// A group of up to 4 TN GEMMs over the same K (a layer's weight gradients), one launch: item
// lin belongs to GEMM g with item0[g] <= lin < item0[g + 1]; every GEMM uses the launch's K
// split length kps, so all items are equally long (gemm4_k's GRP).
struct TnGemm {
  const bf16* A;
  const bf16* B;
  float* C;
  long long slab_stride;
  int M, N, lda, ldb, ldc, tiles_m, tiles_n, item0;
  unsigned a_bytes, b_bytes, c_bytes, pad;
  // the second buffers of rows (a chunked step's other ping-pong chunk: K rows past k_switch)
  const bf16* A2;
  const bf16* B2;
  int lda2, ldb2;
  unsigned a2_bytes, b2_bytes;
};
struct TnGroup {
  int n, total;
  int k_switch;   // the first buffers' rows padded to whole splits (0x7fffffff: one buffer)
  int k0;         // the first buffers' rows (0x7fffffff: one buffer)
  TnGemm d[4];
};

template <int BN>
__device__ __forceinline__ Item decode(int lin, int nwg, int tiles_m, int tiles_n, int group_m, int K, int kps,
                                       int k_switch) {
  Item it;
  it.split = lin / nwg;
  const int wg = lin - it.split * nwg;
  const int per_group = group_m * tiles_n;
  const int gid = wg / per_group;
  const int first_m = gid * group_m;
  const int gsz = min(tiles_m - first_m, group_m);
  const int r = wg - gid * per_group;
  it.m0 = (first_m + r % gsz) * 256;
  it.n0 = (r / gsz) * BN;
  it.kb = it.split * kps;
  it.ke = min(K, it.kb + kps);
  KASSERT(it.m0 < tiles_m * 256 && it.n0 < tiles_n * BN && it.kb <= K,
               "item %d -> tile (%d, %d) k %d", lin, it.m0, it.n0, it.kb);
  it.sel = 0;
  it.g = 0;
  it.role = 0;
  if (it.kb >= k_switch) {
    it.sel = 1;
    it.kb -= k_switch;
    it.ke -= k_switch;
  }
  return it;
}

// 32-deep steps of an item, rounded up to an even count (the two fragment register sets
// alternate statically; a trailing step past the K range reads zeros).
__device__ __forceinline__ int nsteps(const Item& it) {
  const int n = max(1, (it.ke - it.kb + 31) / 32);
  return (n + 1) & ~1;
}

// Epilogue of one item.  OUT 0: bias (+ RoPE) in fp32, bf16; v_permlane16_swap pairs two
// 16-column tiles so each lane holds 8 consecutive columns and writes them with ONE 16-byte
// buffer store (16 rows x 64 contiguous bytes per instruction; the two halves of a row's
// 128-byte line are written by consecutive instructions).  OUT 1: fp32, each lane's 4 columns
// per tile as one 16-byte store.  Exactly STORES (4 / 8 per 16-row block at BN 256, 3 / 6 at
// 192) buffer stores per wave (out-of-range lanes get an offset past the descriptor), which
// the next item's first wait counts.  The wave's tile is 128 x BN/2 (NJ = BN/32 16-column
// tiles); RoPE only at BN 256 (a 64-wide head never straddles two waves there).
// Straight-line code: the lane's bias values are read from LDS once per item (HAS_BIAS is a
// template flag, no per-tile branch or LDS wait), store offsets are 32-bit selects (the C span
// fits the descriptor, so row * ldc cannot overflow), and the RoPE rows' positions and
// cos / sin values are loaded one 16-row block ahead of their use.
__device__ __forceinline__ float silu_ref(float g) { return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)); }

// fp32 epilogue of the 32x32x16 accumulators (M32): lane l holds row l & 31 of each 32 x 32
// block, columns 8 G + 4 (l >> 5) + 0..3 in registers 4G..4G+3: one 16-byte store each, 64 per
// wave (as the 16x16 form's OUT 1).
__device__ __forceinline__ void epilogue_f32_m32(const Item& ci, void* C, int M, int N, int ldc,
                                                 long long slab_stride, unsigned c_bytes, int wm, int wn, int l) {
  acc_drain();
  char* cbase = reinterpret_cast<char*>(C) + (long long)ci.split * slab_stride * 4;
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void*)cbase, (short)0, (int)c_bytes, 0x00020000);
  const int row0 = ci.m0 + wm * 128 + (l & 31);
  const int col0 = ci.n0 + wn * 128 + 4 * (l >> 5);
  static_for<0, 4>([&](auto I) {
    constexpr int bi = decltype(I)::value;
    const int m = row0 + 32 * bi;
    const bool mok = m < M;
    const unsigned rbase = (unsigned)(mok ? m : 0) * (unsigned)ldc * 4u;
    static_for<0, 4>([&](auto J) {
      constexpr int bj = decltype(J)::value;
      static_for<0, 4>([&](auto G) {
        constexpr int gg = decltype(G)::value;
        const int n = col0 + 32 * bj + 8 * gg;
        const unsigned off = (mok && n < N) ? rbase + (unsigned)n * 4u : kOOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc32_read<bi, bj, gg>()), rc, off, 0, 0);
      });
    });
  });
}

// bf16 epilogue of the 32x32x16 accumulators (M32, OUT 0, + fp32 bias): lane l holds row l & 31
// of each 32 x 32 block, columns 8 G + 4 h + 0..3 (h = l >> 5) in registers 4G..4G+3.  Per
// register-group pair (2 g2, 2 g2 + 1) two v_permlane32_swap (lanes 32-63 of the first operand
// trade with lanes 0-31 of the second) leave lane l < 32 with columns 16 g2 + 0..7 and lane
// l + 32 with 16 g2 + 8..15: one 16-byte store each, 32 per wave (as the 16x16 form's OUT 0).
template <bool HAS_BIAS, int SA>
__device__ __forceinline__ void epilogue_bf16_m32(const char* bias_lds, const Item& ci, void* C, int M, int N,
                                                  int ldc, unsigned c_bytes, int wm, int wn, int l) {
  acc_drain();
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(C, (short)0, (int)c_bytes, 0x00020000);
  const int h = l >> 5;
  const int row0 = ci.m0 + wm * 128 + (l & 31);
  const int col0 = ci.n0 + wn * 128 + 8 * h;
  static_for<0, 4>([&](auto I) {
    constexpr int bi = decltype(I)::value;
    const int m = row0 + 32 * bi;
    const bool mok = m < M;
    const unsigned rbase = (unsigned)(mok ? m : 0) * (unsigned)ldc * 2u;
    static_for<0, 4>([&](auto J) {
      constexpr int bj = decltype(J)::value;
      static_for<0, 2>([&](auto G2) {
        constexpr int g2 = decltype(G2)::value;
        f32x4 x = acc32_read<bi, bj, 2 * g2>(), y = acc32_read<bi, bj, 2 * g2 + 1>();
        if constexpr (HAS_BIAS) {
          x += *reinterpret_cast<const f32x4*>(bias_lds + 4 * (32 * bj + 16 * g2 + 4 * h));
          y += *reinterpret_cast<const f32x4*>(bias_lds + 4 * (32 * bj + 16 * g2 + 8 + 4 * h));
        }
        const bf16x4 xo = {(bf16)x[0], (bf16)x[1], (bf16)x[2], (bf16)x[3]};
        const bf16x4 yo = {(bf16)y[0], (bf16)y[1], (bf16)y[2], (bf16)y[3]};
        const u32x2 xd = __builtin_bit_cast(u32x2, xo), yd = __builtin_bit_cast(u32x2, yo);
        const auto s0 = __builtin_amdgcn_permlane32_swap(xd[0], yd[0], false, false);
        const auto s1 = __builtin_amdgcn_permlane32_swap(xd[1], yd[1], false, false);
        const u32x4 w = {s0[0], s1[0], s0[1], s1[1]};
        const int n = col0 + 32 * bj + 16 * g2;
        const unsigned off = (mok && n < N) ? rbase + (unsigned)n * 2u : kOOB;
        __builtin_amdgcn_raw_buffer_store_b128(w, rc, off, 0, SA);
      });
    });
  });
}

// Stream-K, first K half (SK role 1): the wave's 128 x 128 fp32 partial, lane-linear (store
// (i, j) of lane l at ((8 i + j) 64 + l) 16 bytes), written through to memory, drained, then
// the wave's flag.
__device__ __forceinline__ void epilogue_sk_part(const SkArgs& sk, int e, int wave, int l) {
  acc_drain();
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(sk.part + ((long long)e * 4 + wave) * 16384), (short)0, 65536, 0x00020000);
  static_for<0, 8>([&](auto I) {
    constexpr int i = decltype(I)::value;
    static_for<0, 8>([&](auto J) {
      constexpr int j = decltype(J)::value;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc_read<i, j>()), rp,
                                             (unsigned)(((8 * i + j) * 64 + l) * 16), 0, kAuxSys);
    });
  });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (l == 0 && !sk.starve) __hip_atomic_store(sk.flags + e * 4 + wave, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Stream-K, second K half (SK role 2): wait (bounded) for the first half's partial.
__device__ __forceinline__ void sk_wait(const SkArgs& sk, int e, int wave, int l) {
  const unsigned* f = sk.flags + e * 4 + wave;
  const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + 200000000ull;   // 2 s at 100 MHz
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 1u) {
    __builtin_amdgcn_s_sleep(2);
    if (__builtin_amdgcn_s_memrealtime() > deadline) {
      if (l == 0) __hip_atomic_store(sk.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");   // (the partial's loads stay below)
}

// PART (stream-K role 2): the first K half's fp32 partial (epilogue_sk_part's layout, base
// `part` of this wave) is added to the accumulators before bias / RoPE / bf16; block i + 1's
// 8 vectors are loaded (L2-bypassing) under block i's conversions and stores.
template <int OUT, int BN, int ROPE, bool HAS_BIAS, bool SWIGLU = false, int SA = 0, bool PART = false>
__device__ __forceinline__ void epilogue(const char* bias_lds, const Item& ci, void* C, const Rope& rope, int M,
                                         int N, int ldc, long long slab_stride, unsigned c_bytes, int wm, int wn,
                                         int l, const SwiOut& swo = SwiOut{}, const float* part = nullptr) {
  constexpr int NJ = BN / 32;
  const int g = l >> 4;
  const int wcol0 = ci.n0 + wn * (BN / 2);
  const int row0 = ci.m0 + wm * 128 + (l & 15);
  acc_drain();
  if constexpr (OUT == 0) {
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(C, (short)0, (int)c_bytes, 0x00020000);
    const int colg = 16 * (g & 1) + 8 * (g >> 1);
    f32x4 bv[NJ];
    if constexpr (HAS_BIAS) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) bv[j] = *reinterpret_cast<const f32x4*>(bias_lds + 64 * j + 16 * g);
    }
    // RoPE (head_dim ROPE = 64 / 128): rotate-half pairs (d, d + hd/2) live in the same lane,
    // tiles j and j + HJ.  One set of table registers: block i+1's values are loaded right
    // after block i's rotation consumed them, under block i's conversions and stores.
    constexpr int HD = (BN == 256) ? ROPE : 0;
    constexpr int HJ = HD ? HD / 32 : 1;   // tiles per half head: 2 (hd 64) or 4 (hd 128)
    const bool do_rope = HD && rope.cols > 0 && wcol0 < rope.cols;
    f32x4 cs[HJ], sn[HJ];
    auto rope_load = [&](int i) {
      const int m = row0 + 16 * i;
      const long long pp = m < M ? rope.pos[m] : 0;
      KASSERT(m >= M || pp >= 0, "rope position %lld at row %d", pp, m);
      const float* tr = rope.tab + pp * HD;
#pragma unroll
      for (int jh = 0; jh < HJ; ++jh) {
        cs[jh] = *reinterpret_cast<const f32x4*>(tr + 16 * jh + 4 * g);
        sn[jh] = *reinterpret_cast<const f32x4*>(tr + HD / 2 + 16 * jh + 4 * g);
      }
    };
    if constexpr (HD != 0) {
      if (do_rope) rope_load(0);
    }
    const __amdgpu_buffer_rsrc_t rp =
        __builtin_amdgcn_make_buffer_rsrc((void*)part, (short)0, PART ? 65536 : 0, 0x00020000);
    f32x4 pa[PART ? 8 : 1];
    if constexpr (PART) {
      static_assert(BN == 256, "stream-K partials: 256-wide tiles");
#pragma unroll
      for (int j = 0; j < 8; ++j)
        pa[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rp, (unsigned)((j * 64 + l) * 16), 0, kAuxSys));
    }
    static_for<0, 8>([&](auto I) {
      constexpr int i = decltype(I)::value;
      f32x4 v[8];
      f32x4 pc[PART ? 8 : 1];
      if constexpr (PART) {
#pragma unroll
        for (int j = 0; j < 8; ++j) pc[j] = pa[j];
        if constexpr (i + 1 < 8) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            pa[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                  rp, (unsigned)(((8 * (i + 1) + j) * 64 + l) * 16), 0, kAuxSys));
        }
      }
      static_for<0, NJ>([&](auto J) {
        constexpr int j = decltype(J)::value;
        v[j] = acc_read<i, j>();
        if constexpr (PART) v[j] += pc[j];
        if constexpr (HAS_BIAS) v[j] += bv[j];
      });
      const int m = row0 + 16 * i;
      if constexpr (HD != 0) {
        if (do_rope) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int jh = j % (2 * HJ);
            if (jh < HJ && wcol0 + 16 * j < rope.cols) {
              const f32x4 x1 = v[j], x2 = v[j + HJ];
              v[j] = x1 * cs[jh] - x2 * sn[jh];
              v[j + HJ] = x2 * cs[jh] + x1 * sn[jh];
            }
          }
          if (i + 1 < 8) rope_load(i + 1);
        }
      }
      const bool mok = m < M;
      const unsigned rbase = (unsigned)(mok ? m : 0) * (unsigned)ldc * 2u;
      if constexpr (SWIGLU) {
        // h of this lane's 16 gate / up pairs -> 2 stores (exactly, every 16-row block)
        const __amdgpu_buffer_rsrc_t rh =
            __builtin_amdgcn_make_buffer_rsrc((void*)swo.h, (short)0, (int)swo.h_bytes, 0x00020000);
        const unsigned hbase = (unsigned)(mok ? m : 0) * (unsigned)swo.ldh * 2u;
        f32x4 hv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float gg = (float)(bf16)v[j][e], uu = (float)(bf16)v[j + 4][e];
            hv[j][e] = silu_ref(gg) * uu;
          }
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          const bf16x4 o0 = {(bf16)hv[2 * jp][0], (bf16)hv[2 * jp][1], (bf16)hv[2 * jp][2], (bf16)hv[2 * jp][3]};
          const bf16x4 o1 = {(bf16)hv[2 * jp + 1][0], (bf16)hv[2 * jp + 1][1], (bf16)hv[2 * jp + 1][2],
                             (bf16)hv[2 * jp + 1][3]};
          const u32x2 d = __builtin_bit_cast(u32x2, o0), e = __builtin_bit_cast(u32x2, o1);
          const auto sx = __builtin_amdgcn_permlane16_swap(d[0], e[0], false, false);
          const auto sy = __builtin_amdgcn_permlane16_swap(d[1], e[1], false, false);
          const u32x4 w = {sx[0], sy[0], sx[1], sy[1]};
          const int hn = (wcol0 >> 1) + 32 * jp + colg;
          const unsigned off = (mok && 2 * hn < N) ? hbase + (unsigned)hn * 2u : kOOB;
          __builtin_amdgcn_raw_buffer_store_b128(w, rh, off, 0, 0);
        }
      }
#pragma unroll
      for (int jp = 0; jp < NJ / 2; ++jp) {
        const bf16x4 o0 = {(bf16)v[2 * jp][0], (bf16)v[2 * jp][1], (bf16)v[2 * jp][2], (bf16)v[2 * jp][3]};
        const bf16x4 o1 = {(bf16)v[2 * jp + 1][0], (bf16)v[2 * jp + 1][1], (bf16)v[2 * jp + 1][2],
                           (bf16)v[2 * jp + 1][3]};
        const u32x2 d = __builtin_bit_cast(u32x2, o0), e = __builtin_bit_cast(u32x2, o1);
        const auto sx = __builtin_amdgcn_permlane16_swap(d[0], e[0], false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(d[1], e[1], false, false);
        const u32x4 w = {sx[0], sy[0], sx[1], sy[1]};
        const int n = wcol0 + 32 * jp + colg;
        const unsigned off = (mok && n < N) ? rbase + (unsigned)n * 2u : kOOB;
        __builtin_amdgcn_raw_buffer_store_b128(w, rc, off, 0, SA);
      }
    });
  } else {
    char* cbase = reinterpret_cast<char*>(C) + (long long)ci.split * slab_stride * 4;
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void*)cbase, (short)0, (int)c_bytes, 0x00020000);
    static_for<0, 8>([&](auto I) {
      constexpr int i = decltype(I)::value;
      const int m = row0 + 16 * i;
      const bool mok = m < M;
      const unsigned rbase = (unsigned)(mok ? m : 0) * (unsigned)ldc * 4u;
      static_for<0, NJ>([&](auto J) {
        constexpr int j = decltype(J)::value;
        const int n = wcol0 + 16 * j + 4 * g;
        const unsigned off = (mok && n < N) ? rbase + (unsigned)n * 4u : kOOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc_read<i, j>()), rc, off, 0, 0);
      });
    });
  }
}

template <int R>
__device__ __forceinline__ float ror16(float x) {   // value of lane (l + R) % 16 of the same 16-lane row
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x120 + R, 0xF, 0xF, false));
}

// asm-issued 16-byte buffer load: invisible to hipcc's vmcnt bookkeeping (which would drain the
// next item's in-flight LDS-DMA stages at the first use); waited by `pin_vm` with an explicit
// count.
__device__ __forceinline__ u32x4 ld16_asm(__amdgpu_buffer_rsrc_t r, unsigned off) {
  u32x4 v;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(r));
  return v;
}

template <int N_>
__device__ __forceinline__ void pin_vm(u32x4& g, u32x4& u) {
  asm volatile("s_waitcnt vmcnt(%2)" : "+v"(g), "+v"(u) : "n"(N_));
}

// DPP within 8-lane halves of a 16-lane row: lane i <-> 7 - i, and quad lane xor 2 / xor 1.
__device__ __forceinline__ float dpp_half_mirror(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x141, 0xF, 0xF, false));
}
template <int P>
__device__ __forceinline__ float dpp_quad(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), P, 0xF, 0xF, false));
}

// SWB epilogue of one item: 8 blocks of 16 rows.  Loads roll per column group jp, SWB_D (2)
// blocks ahead: block i+2's gate / up vectors of group jp are issued into the register set
// block i has just consumed, so two sets of 8 vectors are live (two blocks of HBM latency
// hidden instead of one) and every wait has a static count (swb_younger; 28 younger VMEM ops
// in steady state).  Column sums: per block, lanes l and l + 8 of a DPP row add their values (row_ror 8);
// lanes 0-7 of the row keep the gate sums, lanes 8-15 the up sums (32 accumulators per lane,
// not 64); at the item's end a mirror / quad butterfly sums each 8-lane half and lanes 0 / 8 of
// every row write the 32 + 32 column partials (fixed order: deterministic).
// Exactly 8 * 8 + 8 stores per wave (out-of-range lanes get an offset past the descriptor).
constexpr int SWB_STORES = 8 * 8 + 8;
// v = x + s (s wave-uniform) as an opaque instruction: hipcc cannot precompute every block's
// offsets ahead of the unrolled epilogue (which would hold 64 of them in VGPRs at once).
__device__ __forceinline__ unsigned opaque_add(unsigned x, unsigned s) {
  unsigned r;
  asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "v"(x), "s"(s));
  return r;
}

// acc += mine + (other of lane (l + 8) % 16 of the DPP row), as volatile asm: ordered with the
// epilogue's other asm (hipcc otherwise sinks the whole accumulation chain to the end of the
// unrolled epilogue and keeps every block's operands live).  s_nop 1: the DPP read of a VGPR
// written by the VALU just before needs two wait states (not inserted for inline asm).
__device__ __forceinline__ void acc_pair(float& acc, float mine, float other) {
  asm volatile("s_nop 1\n\tv_add_f32_dpp %1, %2, %1 row_ror:8 row_mask:0xf bank_mask:0xf\n\tv_add_f32 %0, %0, %1"
               : "+v"(acc), "+v"(mine)
               : "v"(other));
}

// Row blocks of gate / up loads in flight in the SWB epilogue, and the count of VMEM ops a
// wave issues after the two loads of step s = (block s / 4, group s % 4): the prologue loads
// the first SWB_D blocks; step t then issues 2 stores and, while block t / 4 + SWB_D exists,
// the 2 loads of (t / 4 + SWB_D, t % 4) into the set block t / 4 used.
constexpr int swb_ops(int D, int t) { return 2 + (t / 4 + D <= 7 ? 2 : 0); }
constexpr int swb_younger(int D, int s) {
  int n = 0;
  if (s / 4 < D) {
    n = 8 * D - 1 - (2 * s + 1);   // prologue loads after this group's U load
    for (int t = 0; t < s; ++t) n += swb_ops(D, t);
  } else {
    for (int t = s - 4 * D + 1; t < s; ++t) n += swb_ops(D, t);
  }
  return n;
}
static_assert(swb_younger(2, 0) == 14 && swb_younger(2, 31) == 14 && swb_younger(2, 12) == 28, "SWB vmcnt schedule");
static_assert(swb_younger(1, 0) == 6 && swb_younger(1, 8) == 12 && swb_younger(1, 31) == 6, "SWB vmcnt schedule");

template <int SWB_D>
__device__ __forceinline__ void epilogue_swb(const Item& ci, int M, int F, const SwiBwd& sb, int wm, int wn, int l) {
  const int g = l >> 4;
  const int wcol0 = ci.n0 + wn * 128;
  const int row0 = ci.m0 + wm * 128 + (l & 15);
  const int colg = 16 * (g & 1) + 8 * (g >> 1);
  const bool upper = (l & 8) != 0;   // lanes 8-15 of the DPP row accumulate the up sums
  acc_drain();
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)sb.gu, (short)0, (int)sb.gu_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)sb.dgu, (short)0, (int)sb.dgu_bytes, 0x00020000);
  const int c0 = wcol0 + colg;            // this lane's first natural column (jp = 0)
  // gate / up byte offsets of column group jp within a gu row: jp adds 32 columns, which in
  // the interleaved layout is 64 elements when the group crosses into the next 64-block pair
  const unsigned gcol0 = (unsigned)(sb.perm ? ((c0 >> 6) << 7) + (c0 & 63) : c0) * 2u;
  const unsigned uadd = (unsigned)(sb.perm ? 64 : F) * 2u;
  const unsigned gstride = (unsigned)sb.ldgu * 32u, dstride = (unsigned)sb.lddgu * 32u;   // 16 rows
  unsigned goff = (unsigned)row0 * (unsigned)sb.ldgu * 2u + gcol0;   // block 0, group 0 (gate)
  unsigned doff = (unsigned)row0 * (unsigned)sb.lddgu * 2u + (unsigned)c0 * 2u;
  // gate / up vectors of the next SWB_D row blocks in flight (32 VGPRs per set)
  u32x4 G[SWB_D][4], U[SWB_D][4];
  float acc[4][8];
#pragma unroll
  for (int jp = 0; jp < 4; ++jp)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[jp][e] = 0.f;
  // column group jp of a row: natural column c0 + 32 jp; interleaved: + 64 jp elements (c0 and
  // c0 + 32 jp share the 64-column block parity: 32 jp < 128, and (c0 & 63) + 32 jp stays in
  // one gate block only for jp even -> use the exact mapping)
  auto gdelta = [&](int jp) -> unsigned {
    if (!sb.perm) return (unsigned)(32 * jp) * 2u;
    const int c = c0 + 32 * jp;
    return (unsigned)(((c >> 6) << 7) + (c & 63)) * 2u - gcol0;
  };
  auto load = [&](int set, int m, unsigned base, int jp) __attribute__((always_inline)) {
    const bool ok = m < M && c0 + 32 * jp < F;
    const unsigned o = base + gdelta(jp);
    G[set][jp] = ld16_asm(rg, ok ? o : kOOB);
    U[set][jp] = ld16_asm(rg, ok ? o + uadd : kOOB);
  };
  unsigned gahead = goff;   // gu offset of the next block to load
#pragma unroll
  for (int bb = 0; bb < SWB_D; ++bb) {
#pragma unroll
    for (int jp = 0; jp < 4; ++jp) load(bb, row0 + 16 * bb, gahead, jp);
    gahead = opaque_add(gahead, gstride);
  }
  static_for<0, 8>([&](auto I) __attribute__((always_inline)) {
    constexpr int i = decltype(I)::value;
    constexpr int set = i % SWB_D;
    const int m = row0 + 16 * i;
    const bool mok = m < M;
    const unsigned gload = gahead;   // block i + SWB_D
    static_for<0, 4>([&](auto JP) __attribute__((always_inline)) {
      constexpr int jp = decltype(JP)::value;
      // VMEM ops younger than (block i, group jp)'s two loads
      constexpr int YOUNGER = swb_younger(SWB_D, 4 * i + jp);
      pin_vm<YOUNGER>(G[set][jp], U[set][jp]);
      const f32x4 v0 = acc_read<i, 2 * jp>(), v1 = acc_read<i, 2 * jp + 1>();
      const bf16x4 o0 = {(bf16)v0[0], (bf16)v0[1], (bf16)v0[2], (bf16)v0[3]};
      const bf16x4 o1 = {(bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]};
      const u32x2 d2 = __builtin_bit_cast(u32x2, o0), e2 = __builtin_bit_cast(u32x2, o1);
      const auto sx = __builtin_amdgcn_permlane16_swap(d2[0], e2[0], false, false);
      const auto sy = __builtin_amdgcn_permlane16_swap(d2[1], e2[1], false, false);
      const u32x4 w = {sx[0], sy[0], sx[1], sy[1]};
      const bf16x8 dv = __builtin_bit_cast(bf16x8, w);
      const bf16x8 gv = __builtin_bit_cast(bf16x8, G[set][jp]);
      const bf16x8 uv = __builtin_bit_cast(bf16x8, U[set][jp]);
      bf16x8 og, ou;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = (float)dv[e], gg = (float)gv[e], uu = (float)uv[e];
        const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-gg));
        const float a = d * uu * sg * (1.f + gg * (1.f - sg));
        const float b = d * gg * sg;
        og[e] = (bf16)a;
        ou[e] = (bf16)b;
        // lanes l, l + 8 (rows r, r + 8): lower half keeps gate pair sums, upper half up
        const float mine = upper ? b : a, other = upper ? a : b;
        acc_pair(acc[jp][e], mine, other);
      }
      const bool ok = mok && c0 + 32 * jp < F;
      const unsigned od = doff + (unsigned)(64 * jp);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, og), rd, ok ? od : kOOB, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, ou), rd, ok ? od + (unsigned)F * 2u : kOOB, 0, 0);
      if constexpr (i + SWB_D < 8) load(set, m + 16 * SWB_D, gload, jp);
    });
    if constexpr (i + SWB_D < 8) gahead = opaque_add(gahead, gstride);
    if constexpr (i + 1 < 8) doff = opaque_add(doff, dstride);
  });
#pragma unroll
  for (int jp = 0; jp < 4; ++jp)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float a = acc[jp][e];
      a += dpp_half_mirror(a);
      a += dpp_quad<0x4E>(a);   // quad_perm [2, 3, 0, 1]: xor 2
      a += dpp_quad<0xB1>(a);   // quad_perm [1, 0, 3, 2]: xor 1
      acc[jp][e] = a;
    }
  const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc((void*)sb.part, (short)0, (int)sb.part_bytes, 0x00020000);
  const unsigned pbase = (unsigned)((ci.m0 >> 7) + wm) * (unsigned)(2 * F) * 4u;
  const bool writer = (l & 7) == 0;    // lane 0 (gate) and lane 8 (up) of every DPP row
#pragma unroll
  for (int jp = 0; jp < 4; ++jp) {
    const int c = c0 + 32 * jp + (upper ? F : 0);
    const bool ok = writer && c0 + 32 * jp < F;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 v = {acc[jp][4 * h], acc[jp][4 * h + 1], acc[jp][4 * h + 2], acc[jp][4 * h + 3]};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rp,
                                             ok ? pbase + (unsigned)(c + 4 * h) * 4u : kOOB, 0, 0);
    }
  }
}

// OUT: 0 = bf16 C (+ fp32 bias[n], + RoPE); 1 = fp32 C / split-K slab.
// DIAG: 0 = production; 1 / 2 = the timing builds (per-wave s_memtime split; 2 without DMA);
// 3 = the ablation build that reads `dbg` (timing-only, tools/gemm4_probe.py): 4 = no DMA
// wait, 8 = no step barrier.  Only DIAG 3 tests dbg, so the production step has no runtime
// branch on it.
// FAST (every item's K range a multiple of 64, so no step reads past K): the DMA stream
// advances the buffer descriptors' base address and record count by SALU once per stage
// (hipBLASLt's form) and every piece reuses its per-item lane offset: no VALU, no per-lane
// K check in front of a DMA piece; rows past M / N still land past the record count.
// SCHED 1: the stage's DMA pieces one per MFMA row (rows 0-7) instead of two per row in rows
// 4-7.
// BN: tile columns, 256 (waves 128 x 128) or 192 (waves 128 x 96: the N = 768 projections
// become 512 tiles, two per CU, instead of 384 = 1.5 per CU).  Per stage a wave issues NQ =
// 4 + BN/64 DMA pieces (4 of A, 4 or 3 of B).
// ROPE (head_dim 64 / 128, 0 = none): the RoPE epilogue is compiled in (QKV projection only:
// its code and register pressure stay out of the plain kernels).
// SWIGLU: the gate|up form (SwiOut).
// BR: rows of MFMAs (NJ each) a step issues BEFORE its DMA wait + barrier.  0 = the barrier
// opens the step.  BR > 0: the step's first rows run on fragments already in registers, the
// wave reaches the barrier with MFMAs in flight and the next-step fragment reads follow it
// (rows BR .. BR + 3), so the barrier / wait time overlaps matrix work instead of draining
// the pipe once per 32-deep step.  (Safe: the DMA a step issues writes the slot read two
// steps earlier, retired before the previous step's barrier.)
// M32: the 32x32x16 MFMA main loop (TN only: both operands MN-major, fp32 out, 256-wide):
// 32 MFMAs of 32 cycles per 32-deep step instead of 64 of 16 -- half the MFMA issue slots and
// half the operand-register reads per FLOP, so the step's 32 transposed reads, 8 DMA pieces and
// address / SALU work fit in the MFMA shadow (the 16x16x32 TN step issues ~1.5k cycles of
// non-MFMA work against 1024 of matrix time).
template <bool AK, bool BKM, int OUT, int DIAG = 0, bool FAST = false, int SCHED = 0, int BN = 256, int ROPE = 0,
          bool SWIGLU = false, int SWB = 0, int BR = 0, int SA = 0, bool M32 = false, bool GRP = false,
          bool SK = false>
__global__ __launch_bounds__(256, 1) void gemm4_k(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                  void* __restrict__ C, const float* __restrict__ bias, int M, int N,
                                                  int K, int lda, int ldb, int ldc, int kps, int splits,
                                                  long long slab_stride, unsigned a_bytes, unsigned b_bytes,
                                                  unsigned c_bytes, Rope rope, int group_m, Dual dual, int dbg,
                                                  unsigned long long* diag, SwiOut swo = SwiOut{},
                                                  SwiBwd swb = SwiBwd{}, TnGroup grp = TnGroup{},
                                                  SkArgs sk = SkArgs{}) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_TOTAL];
  constexpr bool TIMED = DIAG == 1 || DIAG == 2;   // the s_memtime builds
  constexpr int NJ = BN / 32;                  // 16-column MFMA tiles per wave
  constexpr int NBQ = BN / 64;                 // B pieces per wave per stage
  constexpr int NQ = 4 + NBQ;                  // DMA pieces per wave per stage
  // store instructions per wave per item (+ the SwiGLU output's 2 per 16-row block)
  constexpr int STORES = SWB ? SWB_STORES : (OUT == 0 ? 4 * NJ : 8 * NJ) + (SWIGLU ? 16 : 0);
  static_assert(!SWIGLU || (OUT == 0 && BN == 256 && ROPE == 0), "SwiGLU epilogue: bf16 256-wide tiles");
  static_assert(!SWB || (OUT == 0 && BN == 256 && ROPE == 0 && !SWIGLU), "SwiGLU-backward epilogue: bf16 256-wide tiles");
  static_assert(BN == 256 || BN == 192, "tile width");
  static_assert(BR >= 0 && BR <= 4 && (BR == 0 || DIAG == 0), "barrier row");
  static_assert(!M32 || ((AK ? true : (!BKM && OUT == 1)) && BN == 256 && SCHED == 1 && ROPE == 0 &&
                          !SWIGLU && !SWB),
                "32x32x16 main loop: TN fp32, NN / NT fp32 or bf16 (+ bias), 256-wide");
  static_assert(!GRP || (M32 && FAST), "grouped TN: the 32x32x16 FAST kernel");
  static_assert(!SK || (AK && OUT == 0 && BN == 256 && FAST && SCHED == 1 && BR == 0 && ROPE == 0 && !SWIGLU && !SWB &&
                        !M32 && !GRP && DIAG == 0),
                "stream-K: plain bf16 NT / NN, 256-wide FAST kernel");
  // ring pieces issued before the step's barrier (their count joins the wait, and the bias
  // DMA issued after the barrier has NQ - PBB younger ring pieces)
  constexpr int PBB = SCHED == 1 ? (BR < NQ ? BR : NQ) : 0;

  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + 255) / 256;
  const int nwg = tiles_m * tiles_n;
  const int total = GRP ? grp.total : (SK ? 2 * (int)gridDim.x : nwg * splits);
  // work item -> tile / K range (GRP: of its GEMM in the group)
  auto gdecode = [&](int lin) -> Item {
    if constexpr (SK) {
      const int Gs = gridDim.x, E = sk.extra;
      const bool second = lin >= Gs;
      const int c = second ? lin - Gs : lin;
      int tile, role;
      if (c < E) {
        tile = second ? c : Gs + c;
        role = second ? 0 : 1;
      } else {
        tile = second ? Gs + c - E : c;
        role = second ? 2 : 0;
      }
      Item x = decode<BN>(tile, nwg, tiles_m, tiles_n, group_m, K, K, 0x7fffffff);
      x.role = role;
      x.g = tile - Gs;   // (roles 1 / 2: the extra tile's index e, its partial / flag slot)
      const int kh = K >> 1;   // (K % 128 == 0: both halves whole 64-deep stages)
      if (role == 1) x.ke = kh;
      if (role == 2) x.kb = kh;
      return x;
    } else if constexpr (GRP) {
      int g = 0;
#pragma unroll
      for (int i = 1; i < 4; ++i)
        if (i < grp.n && lin >= grp.d[i].item0) g = i;
      const TnGemm& d = grp.d[g];
      Item x = decode<BN>(lin - d.item0, d.tiles_m * d.tiles_n, d.tiles_m, d.tiles_n, group_m, K, kps, grp.k_switch);
      x.g = g;
      // a two-buffer group's first buffer is padded to whole splits: its last split ends at the
      // buffer's rows (the padding stages are past nlive: zeros, no record-count underflow)
      if (x.sel == 0 && x.ke > grp.k0) x.ke = grp.k0;
      return x;
    } else {
      return decode<BN>(lin, nwg, tiles_m, tiles_n, group_m, K, kps, dual.k_switch);
    }
  };
  const int G = gridDim.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int l = lane_id();
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, (int)b_bytes, 0x00020000);
  const bool dual_on = dual.A2 != nullptr;
  const __amdgpu_buffer_rsrc_t ra2 =
      dual_on ? __builtin_amdgcn_make_buffer_rsrc((void*)dual.A2, (short)0, (int)dual.a2_bytes, 0x00020000) : ra;
  const __amdgpu_buffer_rsrc_t rb2 =
      dual_on ? __builtin_amdgcn_make_buffer_rsrc((void*)dual.B2, (short)0, (int)dual.b2_bytes, 0x00020000) : rb;
  const int lda2 = dual_on ? dual.lda2 : lda, ldb2 = dual_on ? dual.ldb2 : ldb;
  const __amdgpu_buffer_rsrc_t rbias =
      __builtin_amdgcn_make_buffer_rsrc((void*)bias, (short)0, bias ? N * 4 : 0, 0x00020000);
  char* bias_lds = smem + RING + wave * 512;

  int it = xcd_remap(blockIdx.x, G);
  if (it >= total) return;

  // ---- producer cursor: the DMA stream runs 3 steps ahead of the consumer, across items.
  int p_it = it;
  Item pi = gdecode(p_it);
  int p_t = 0, p_nk = nsteps(pi);
  int p_slot = 0;
  // Per-item lane offsets of the wave's NQ DMA pieces (4 of A, NBQ of B): a step adds one
  // uniform term per operand and checks the K bound against a lane constant (kpos).  Piece
  // j of an operand covers LDS bytes [1 KiB j, 1 KiB (j + 1)) of its half of the slot; an
  // MN-major image has 2 * (tile extent) bytes per k row (A: 256, B: BN).
  unsigned pbase[8];
  auto rebase = [&]() {
    const bool s2 = pi.sel != 0;
    const int la = GRP ? (s2 ? grp.d[pi.g].lda2 : grp.d[pi.g].lda) : (s2 ? lda2 : lda);
    const int lb = GRP ? (s2 ? grp.d[pi.g].ldb2 : grp.d[pi.g].ldb) : (s2 ? ldb2 : ldb);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const bool isA = q < 4;
      const bool km = isA ? AK : BKM;
      const int j = wave + 4 * (q & 3);
      const int r0 = isA ? pi.m0 : pi.n0;
      const int ld = isA ? la : lb;
      if (km) {
        const int row = 16 * j + (l >> 2);
        const int c = (l & 3) ^ kh(row);
        const int rr = (SWIGLU && !isA) ? gu_nat(r0 + row, N >> 1) : r0 + row;   // (rows < N: N % 128 == 0)
        pbase[q] = (unsigned)(((long long)rr * ld + 8 * c) * 2);
      } else if (isA || BN == 256) {
        const int lin = j * 64 + l;
        const int row = lin >> 5;
        const int c = (lin & 31) ^ (M32 ? m32_swz(row) : (mnh(row) << 1));
        pbase[q] = (unsigned)(((long long)row * ld + r0 + 8 * c) * 2);
      } else {
        const int lin = j * 64 + l;
        const int row = lin / (BN / 8);
        const int c = (lin - row * (BN / 8)) ^ mn_swz<BN>(row);
        pbase[q] = (unsigned)(((long long)row * ld + r0 + 8 * c) * 2);
      }
    }
  };
  auto kpos = [&](int q) -> int {
    const bool km = q < 4 ? AK : BKM;
    const int j = wave + 4 * (q & 3);
    if (km) {
      const int row = 16 * j + (l >> 2);
      return 8 * ((l & 3) ^ kh(row));
    }
    return (q < 4 || BN == 256) ? (j * 64 + l) >> 5 : (j * 64 + l) / (BN / 8);
  };
  rebase();
  // FAST: descriptors of the producer's current stage: the item's stage-0 base / record count
  // and per-stage byte stride are set once per item (item_rsrc), a stage adds p_t strides.
  __amdgpu_buffer_rsrc_t sra = ra, srb = rb;
  unsigned long long ia = 0, ib = 0;   // (integers: pointer-typed captures stay in scratch)
  unsigned na0 = 0, nb0 = 0, sta = 0, stb = 0;
  int nlive = 0;   // stages of the item with k in range (an empty trailing split has none)
  auto item_rsrc = [&]() {
    if constexpr (FAST) {
      const bool s2 = pi.sel != 0;
      const int la = GRP ? (s2 ? grp.d[pi.g].lda2 : grp.d[pi.g].lda) : (s2 ? lda2 : lda);
      const int lb = GRP ? (s2 ? grp.d[pi.g].ldb2 : grp.d[pi.g].ldb) : (s2 ? ldb2 : ldb);
      const long long adv_a = AK ? (long long)pi.kb * 2 : (long long)pi.kb * la * 2;
      const long long adv_b = BKM ? (long long)pi.kb * 2 : (long long)pi.kb * lb * 2;
      const bf16* a0 = GRP ? (s2 ? grp.d[pi.g].A2 : grp.d[pi.g].A) : (s2 ? dual.A2 : A);
      const bf16* b0 = GRP ? (s2 ? grp.d[pi.g].B2 : grp.d[pi.g].B) : (s2 ? dual.B2 : B);
      ia = reinterpret_cast<unsigned long long>(a0) + adv_a;
      ib = reinterpret_cast<unsigned long long>(b0) + adv_b;
      na0 = (GRP ? (s2 ? grp.d[pi.g].a2_bytes : grp.d[pi.g].a_bytes) : (s2 ? dual.a2_bytes : a_bytes)) - (unsigned)adv_a;
      nb0 = (GRP ? (s2 ? grp.d[pi.g].b2_bytes : grp.d[pi.g].b_bytes) : (s2 ? dual.b2_bytes : b_bytes)) - (unsigned)adv_b;
      sta = AK ? 64u : 64u * (unsigned)la;
      stb = BKM ? 64u : 64u * (unsigned)lb;
      nlive = (pi.ke - pi.kb + 31) / 32;
    }
  };
  item_rsrc();
  // (one operand per call: the step places them in the shadow of its first MFMAs, see `step`)
  // (one operand each: the step places them in the shadow of its first two MFMAs)
  auto stage_rsrc_a = [&]() {
    if constexpr (FAST) {
      const unsigned off = (unsigned)p_t * sta;
      const unsigned n = (p_t < nlive && p_it < total) ? na0 - off : 0u;
      sra = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(ia + off), (short)0, (int)n, 0x00020000);
    }
  };
  auto stage_rsrc_b = [&]() {
    if constexpr (FAST) {
      const unsigned off = (unsigned)p_t * stb;
      const unsigned n = (p_t < nlive && p_it < total) ? nb0 - off : 0u;
      srb = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(ib + off), (short)0, (int)n, 0x00020000);
    }
  };
  // DMA piece q (< 8) of the producer's current stage
  auto issue = [&](int q) {
    if constexpr (FAST) {
      if constexpr (DIAG == 2) return;
      dma16(q < 4 ? sra : srb, smem + p_slot * SLOT + (q < 4 ? 0 : 16384) + (wave + 4 * (q & 3)) * 1024, pbase[q]);
      return;
    }
    const bool live = p_it < total;
    const int krem = (live ? pi.ke : 0) - (pi.kb + 32 * p_t);   // valid k in this stage
    const int k0 = pi.kb + 32 * p_t;
    const bool s2 = pi.sel != 0;
    const bool isA = q < 4;
    const bool km = isA ? AK : BKM;
    const unsigned add = km ? (unsigned)(k0 * 2)
                            : (unsigned)((long long)k0 * (isA ? (s2 ? lda2 : lda) : (s2 ? ldb2 : ldb)) * 2);
    const unsigned off = (kpos(q) < krem) ? pbase[q] + add : kOOB;
    if constexpr (DIAG == 2) return;   // timing-only: no DMA issued (stale LDS, wrong results)
    dma16(isA ? (s2 ? ra2 : ra) : (s2 ? rb2 : rb),
          smem + p_slot * SLOT + (isA ? 0 : 16384) + (wave + 4 * (q & 3)) * 1024, off);
  };
  auto advance = [&]() {
    p_slot = (p_slot + 1) & 3;
    if (p_it < total && ++p_t == p_nk) {
      p_it += G;
      p_t = 0;
      if (p_it < total) {
        pi = gdecode(p_it);
        p_nk = nsteps(pi);
        rebase();
        item_rsrc();
      }
    }
  };
#pragma unroll
  for (int s0 = 0; s0 < 3; ++s0) {
    stage_rsrc_a();
    stage_rsrc_b();
#pragma unroll
    for (int q = 0; q < NQ; ++q) issue(q);
    advance();
  }

  Frags<AK, BKM, BN, M32> F0, F1;
  int c_slot = 0;
  // M32: per-lane offsets of the 4 fragment blocks of each MN-major operand in a slot (B:
  // + 16384); a K-major operand's two k-half offsets (its blocks are immediates apart)
  unsigned m32a[4] = {0, 0, 0, 0}, m32b[4] = {0, 0, 0, 0};
  unsigned k32a[2] = {0, 0}, k32b[2] = {0, 0};
  if constexpr (M32) {
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      if constexpr (!AK) m32a[nb] = m32_off(wm * 128, nb, l);
      if constexpr (!BKM) m32b[nb] = 16384u + m32_off(wn * 128, nb, l);
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if constexpr (AK) k32a[kk] = k32_off(wm * 128, kk, l);
      if constexpr (BKM) k32b[kk] = 16384u + k32_off(wn * 128, kk, l);
    }
  }
  // DIAG build only (timing diagnosis, never the production kernel): cycles spent in the
  // step-entry waits + barrier, in the step bodies and in the epilogues, per wave.
  unsigned long long t_wait = 0, t_body = 0, t_epi = 0, t_mark = 0;
  auto stamp = [&]() -> unsigned long long {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
  };
  // fragments of the first step: stage 0 landed (two younger stages of NQ pieces in flight)
  wait_vmcnt<2 * NQ>();
  __builtin_amdgcn_s_barrier();
  read_frags<AK, BKM, BN, M32>(F0, smem, wm, wn, l);
  if constexpr (TIMED) t_mark = stamp();

  // One consumer step on `cur`, prefetching the next step's fragments into `nxt`.
  // Entry wait: stage s+1 landed for this wave (younger: stage s+2 = NQ pieces, plus the
  // previous item's epilogue stores on an item's first step), then the step barrier.
  auto step = [&](Frags<AK, BKM, BN, M32>& cur, Frags<AK, BKM, BN, M32>& nxt, bool first, auto zero, auto nopf, bool last,
                  int bcol0) {
    constexpr bool ZR = decltype(zero)::value;
    constexpr bool NOPF = decltype(nopf)::value;   // no next-step fragment reads (item end, SWB)
    if constexpr (TIMED) {
      const unsigned long long t = stamp();
      t_body += t - t_mark;
      t_mark = t;
    }
    // `cur` was read a whole step ago: retire it here so the MFMAs below need no LDS wait
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
    cur.a.pin();
    cur.b.pin();
    // Stage s+1 landed for this wave (younger: stage s+2 = NQ pieces, the PBB pieces of stage
    // s+3 issued before the barrier, plus the previous item's epilogue stores on an item's
    // first step), then the step barrier; the bias DMA of the item's last step after it.
    auto sync = [&]() __attribute__((always_inline)) {
      if (DIAG == 3 && (dbg & 4)) wait_vmcnt<63>();   // timing-only: no wait for the DMA (wrong results)
      else if (first) wait_vmcnt<(NQ + PBB + STORES < 63 ? NQ + PBB + STORES : 63)>();
      else wait_vmcnt<NQ + PBB>();
      if (!(DIAG == 3 && (dbg & 8))) __builtin_amdgcn_s_barrier();
      if constexpr (TIMED) {
        const unsigned long long t = stamp();
        t_wait += t - t_mark;
        t_mark = t;
      }
      if (OUT == 0 && last && bias) {
        // the epilogue's bias values of this wave (128, of which BN/2 used) into its LDS area
        // by two 256-byte LDS-DMA pieces, ahead of this step's remaining NQ - PBB ring pieces
        // (the epilogue waits vmcnt(NQ - PBB), no barrier: the wave reads only what it loaded)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int n = bcol0 + 64 * h + l;
          const int nb = SWIGLU ? gu_nat(n, N >> 1) : n;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rbias, (__attribute__((address_space(3))) void*)(bias_lds + 256 * h),
                                                   4, n < N ? (unsigned)(nb * 4) : kOOB, 0, 0, 0);
        }
      }
    };
    if constexpr (BR == 0) sync();

    c_slot = (c_slot + 1) & 3;
    const char* src = smem + c_slot * SLOT;
    if constexpr (M32) {
      // 32 MFMAs t = 16 kk + 4 bi + bj; after MFMA t < 16 the next step's fragment t (A for
      // t < 8, B after: two transposed reads each); DMA piece q after MFMA 4 q + 2.  BR > 0:
      // the wait + barrier after MFMA 4 BR - 1 (BR blocks of 4 MFMAs on fragments already in
      // registers ahead of it) and the next step's reads shifted behind it by 4 BR MFMAs.
      static_for<0, 32>([&](auto T) {
        constexpr int t = decltype(T)::value;
        constexpr int kk = t >> 4, bi = (t >> 2) & 3, bj = t & 3;
        constexpr int tr = t - 4 * BR;   // read slot of this MFMA
        acc32_mfma<bi, bj, ZR && kk == 0>(cur.b.get(2 * bj + kk), cur.a.get(2 * bi + kk));
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (t == 0) stage_rsrc_a();
        if constexpr (t == 1) stage_rsrc_b();
        if constexpr (BR > 0 && t == 4 * BR - 1) sync();
        // next step's fragments: block nb of A after MFMA 4 BR + 2 nb, of B after 4 BR + 8 + 2 nb
        if constexpr (!NOPF && tr >= 0 && tr < 8 && (tr & 1) == 0) {
          if constexpr (AK) nxt.a.load_nb(tr >> 1, src + k32a[0], src + k32a[1]);
          else nxt.a.load_nb(tr >> 1, src + m32a[tr >> 1]);
        }
        if constexpr (!NOPF && tr >= 8 && tr < 16 && (tr & 1) == 0) {
          if constexpr (BKM) nxt.b.load_nb((tr - 8) >> 1, src + k32b[0], src + k32b[1]);
          else nxt.b.load_nb((tr - 8) >> 1, src + m32b[(tr - 8) >> 1]);
        }
        if constexpr ((t & 3) == 2 && (t >> 2) < NQ) issue(t >> 2);
        __builtin_amdgcn_sched_barrier(0);
      });
      advance();
    } else {
    // Rows q of NJ MFMAs (A fragment q against every B fragment).  Rows BR .. BR+3 read the
    // next step's fragments (A 2r, 2r+1; B 2r, 2r+1 while < NJ; r = q - BR).  DMA pieces:
    // SCHED 0 two per row in rows 4-7, SCHED 1 one per row.  At NJ = 8 this is the hand-placed
    // order of the 256-wide kernel: MFMA j, then the event after it.
    static_for<0, 8>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      static_for<0, NJ>([&](auto J) {
        constexpr int j = decltype(J)::value;
        acc_mfma<q, j, ZR>(cur.b.get(j), cur.a.get(q));
        __builtin_amdgcn_sched_barrier(0);
        // this step's stage descriptors (scalar work) in the shadow of the first MFMAs
        if constexpr (q == 0 && j == 0) stage_rsrc_a();
        if constexpr (q == 0 && j == 1) stage_rsrc_b();
        if constexpr (BR > 0 && q == BR - 1 && j == NJ - 1) sync();
        constexpr int rq = q - BR;
        if constexpr (rq >= 0 && rq < 4 && !NOPF) {
          // read slots after MFMA 0 / 2 / 4 / 6 (NJ 8) or 0 / 2 / 3 / 5 (NJ 6)
          constexpr int r0 = 0, r1 = 2, r2 = NJ == 8 ? 4 : 3, r3 = NJ == 8 ? 6 : 5;
          if constexpr (j == r0) nxt.a.load(2 * rq, src, wm * 128 + 32 * rq, l);
          if constexpr (j == r1 && 2 * rq < NJ) nxt.b.load(2 * rq, src + 16384, wn * (BN / 2) + 32 * rq, l);
          if constexpr (j == r2) nxt.a.load(2 * rq + 1, src, wm * 128 + 32 * rq + 16, l);
          if constexpr (j == r3 && 2 * rq + 1 < NJ)
            nxt.b.load(2 * rq + 1, src + 16384, wn * (BN / 2) + 32 * rq + 16, l);
        }
        if constexpr (SCHED == 1) {
          if constexpr (j == 3 && q < NQ) issue(q);
        } else if constexpr (q >= 4) {
          constexpr int d0 = 1, d1 = NJ == 8 ? 5 : 4;
          if constexpr (j == d0 && 2 * (q - 4) < NQ) issue(2 * (q - 4));
          if constexpr (j == d1 && 2 * (q - 4) + 1 < NQ) issue(2 * (q - 4) + 1);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    });
    advance();
    }
  };

  for (bool first = true; it < total; it += G, first = false) {
    const Item ci = gdecode(it);
    const int nk = nsteps(ci);
    const int bcol0 = ci.n0 + wn * (BN / 2);
    constexpr std::false_type NO{};
    if constexpr (SK) {
      // As SWB below: the item's last step reads no fragments, so F0 / F1 are dead across the
      // epilogue (the partial-add form holds 16 vectors of the partial); the next item's first
      // fragments are read after it.
      step(F0, F1, !first, std::true_type{}, NO, false, bcol0);
      for (int t = 1; t < nk - 1; t += 2) {
        step(F1, F0, false, NO, NO, false, bcol0);
        step(F0, F1, false, NO, NO, false, bcol0);
      }
      step(F1, F0, false, NO, std::true_type{}, true, bcol0);
      if (ci.role == 1) {
        epilogue_sk_part(sk, ci.g, wave, l);
      } else {
        if (bias) wait_vmcnt<NQ - PBB>();   // this wave's bias DMA landed
        if (ci.role == 2) {
          sk_wait(sk, ci.g, wave, l);
          const float* pw = sk.part + ((long long)ci.g * 4 + wave) * 16384;
          if (bias)
            epilogue<0, 256, 0, true, false, SA, true>(bias_lds, ci, C, rope, M, N, ldc, 0, c_bytes, wm, wn, l, swo, pw);
          else
            epilogue<0, 256, 0, false, false, SA, true>(bias_lds, ci, C, rope, M, N, ldc, 0, c_bytes, wm, wn, l, swo, pw);
        } else if (bias) {
          epilogue<0, 256, 0, true, false, SA>(bias_lds, ci, C, rope, M, N, ldc, 0, c_bytes, wm, wn, l, swo);
        } else {
          epilogue<0, 256, 0, false, false, SA>(bias_lds, ci, C, rope, M, N, ldc, 0, c_bytes, wm, wn, l, swo);
        }
      }
      read_frags<AK, BKM, BN, M32>(F0, smem + c_slot * SLOT, wm, wn, l);
      continue;
    }
    if constexpr (SWB) {
      // The register-hungry SwiGLU-backward epilogue: the item's last step reads no fragments
      // (F0 / F1 are dead across the epilogue); the next item's first-step fragments are read
      // after it from the slot that step would have read (landed at its entry wait, rewritten
      // only by a DMA issued behind the next step's barrier).
      step(F0, F1, !first, std::true_type{}, NO, false, bcol0);
      for (int t = 1; t < nk - 1; t += 2) {
        step(F1, F0, false, NO, NO, false, bcol0);
        step(F0, F1, false, NO, NO, false, bcol0);
      }
      step(F1, F0, false, NO, std::true_type{}, true, bcol0);
      epilogue_swb<SWB>(ci, M, N, swb, wm, wn, l);
      read_frags<AK, BKM, BN, M32>(F0, smem + c_slot * SLOT, wm, wn, l);
      continue;
    }
    step(F0, F1, !first, std::true_type{}, NO, false, bcol0);
    step(F1, F0, false, NO, NO, nk == 2, bcol0);
    for (int t = 2; t < nk; t += 2) {
      step(F0, F1, false, NO, NO, false, bcol0);
      step(F1, F0, false, NO, NO, t + 2 >= nk, bcol0);
    }
    if constexpr (TIMED) {
      const unsigned long long t = stamp();
      t_body += t - t_mark;
      t_mark = t;
    }
    if constexpr (GRP) {
      const TnGemm& d = grp.d[ci.g];
      epilogue_f32_m32(ci, d.C, d.M, d.N, d.ldc, d.slab_stride, d.c_bytes, wm, wn, l);
    } else if constexpr (M32 && OUT == 1) {
      epilogue_f32_m32(ci, C, M, N, ldc, slab_stride, c_bytes, wm, wn, l);
    } else if constexpr (M32) {
      if (bias) {
        wait_vmcnt<NQ - PBB>();   // this wave's bias DMA landed (younger: the ring pieces after it)
        epilogue_bf16_m32<true, SA>(bias_lds, ci, C, M, N, ldc, c_bytes, wm, wn, l);
      } else {
        epilogue_bf16_m32<false, SA>(bias_lds, ci, C, M, N, ldc, c_bytes, wm, wn, l);
      }
    }
    if constexpr (M32) {
      if constexpr (TIMED) {
        const unsigned long long t = stamp();
        t_epi += t - t_mark;
        t_mark = t;
      }
      continue;
    }
    if (OUT == 0 && bias) wait_vmcnt<NQ - PBB>();   // this wave's bias DMA landed (younger: the ring pieces after it)
    if (OUT == 0 && bias)
      epilogue<OUT, BN, ROPE, true, SWIGLU, SA>(bias_lds, ci, C, rope, M, N, ldc, slab_stride, c_bytes, wm, wn, l, swo);
    else
      epilogue<OUT, BN, ROPE, false, SWIGLU, SA>(bias_lds, ci, C, rope, M, N, ldc, slab_stride, c_bytes, wm, wn, l, swo);
    if constexpr (TIMED) {
      const unsigned long long t = stamp();
      t_epi += t - t_mark;
      t_mark = t;
    }
  }
  if constexpr (TIMED) {
    if (l == 0) {
      unsigned long long* d = diag + (blockIdx.x * 4 + wave) * 4;
      d[0] = t_wait;
      d[1] = t_body;
      d[2] = t_epi;
      d[3] = 1;
    }
  }
  // no LDS-DMA may still be writing when the workgroup's LDS is released
  wait_vmcnt<0>();
}

// Split-K reduction of a TN group (gemm4_k GRP): out_g[i] (+)= sum_s ws_g[s][i] for each GEMM g
// of the launch, in a fixed order (deterministic); segment g holds elements [pre[g], pre[g+1])
// of one flat index space (every segment a multiple of 4 long).
struct RedGroup {
  int n, S;
  long long pre[5];
  const float* ws[4];
  float* out[4];
  int acc[4];
};
__global__ __launch_bounds__(256) void splitk_reduce_group_k(RedGroup r) {
  const long long tot = r.pre[r.n];
  for (long long i = (blockIdx.x * (long long)blockDim.x + threadIdx.x) * 4; i < tot;
       i += (long long)gridDim.x * blockDim.x * 4) {
    int g = 0;
#pragma unroll
    for (int k = 1; k < 4; ++k)
      if (k < r.n && i >= r.pre[k]) g = k;
    const long long j = i - r.pre[g], ng = r.pre[g + 1] - r.pre[g];
    float* o = r.out[g] + j;
    f32x4 v = r.acc[g] ? *reinterpret_cast<const f32x4*>(o) : (f32x4){0.f, 0.f, 0.f, 0.f};
    const float* w = r.ws[g] + j;
    for (int k = 0; k < r.S; ++k) v += *reinterpret_cast<const f32x4*>(w + k * ng);
    *reinterpret_cast<f32x4*>(o) = v;
  }
}

}  // namespace g4
}  // namespace dpfs

using namespace dpfs;
using namespace dpfs::g4;

static int g4_cu_count() {
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

static int g_g4_group_m = 4;
// Timing-only ablations (tools/gemm4_probe.py --ablate): bit 1 = output descriptor with zero
// records (every store dropped), bit 2 = operand descriptors with zero records (every DMA
// returns zeros, no memory traffic), 4 = no DMA wait, 8 = no step barrier (wrong results).
// Bits 4 / 8 (and 1024: none) run the DIAG-3 build of the NT 256-wide kernel, the only one
// that reads them.
// Blocks of 4 MFMAs ahead of each step's wait + barrier in the 32x32x16 (TN weight-gradient)
// main loop: 0 (default), 1, 2 (A/B hook).
static int g_g4_br_tn = 0;
extern "C" void dpfs_gemm4_br_tn(int v) { g_g4_br_tn = (v >= 0 && v <= 2) ? v : 0; }
static int g_g4_ablate = 0;
static unsigned long long* g_g4_diag = nullptr;   // [grid][4 waves][wait, body, epilogue, valid]
extern "C" void dpfs_gemm4_ablate(int v) { g_g4_ablate = v; }
extern "C" void dpfs_gemm4_diag(void* p) { g_g4_diag = (unsigned long long*)p; }
// Main-loop variant (tools/gemm4_probe.py A/B): 0 = one DMA piece per MFMA row (default),
// 1 = two pieces per row in rows 4-7; 2 = per-lane K checks even where FAST applies.
static int g_g4_sched = 0;
extern "C" void dpfs_gemm4_sched(int v) { g_g4_sched = v; }
// Rows of MFMAs before each step's barrier (gemm4_k's BR) of the plain FAST kernels: 0, 1, 2.
// 2 (default since the end of round 6): -0.18 ms per training step against 0 in 6 of 6
// same-box interleaved rounds (profiles/r6_gemm_br_ab.txt); 1 is within 0.01 ms of 2.
static int g_g4_br = 2;
extern "C" void dpfs_gemm4_br(int v) { g_g4_br = (v >= 0 && v <= 2) ? v : 0; }
extern "C" void dpfs_gemm4_group_m(int g) { g_g4_group_m = g > 0 ? g : 4; }
// TN main loop: 1 = the 32x32x16 form (gemm4_k's M32, default), 0 = 16x16x32 (A/B probes).
static int g_g4_m32 = 1;
extern "C" void dpfs_gemm4_m32(int v) { g_g4_m32 = v ? 1 : 0; }
// NN / NT main loop on 256-wide tiles: bit 0 = 32x32x16 for the fp32 (split-K) output, bit 1 =
// for the bf16 (+ bias) output; 0 = 16x16x32 (default: the K-major 32x32x16 form measured
// 0.3 ms/step slower in the GPT-2-small step, profiles/r5_m32k_ab.txt)
static int g_g4_m32k = 0;
extern "C" void dpfs_gemm4_m32k(int v) { g_g4_m32k = v & 3; }

// gate|up projection with SwiGLU in the epilogue (SwiOut): C[M, N] = A perm(B)^T + perm(bias)
// (B / bias in the natural [gate | up] layout, read interleaved: reference.gu_perm),
// H[M, N / 2] = silu(gate) * up.  Returns false (nothing launched) where the 256-wide FAST
// kernel does not apply.
extern "C" bool dpfs_gemm4_nt_swiglu(const void* A, const void* B, void* C, const float* bias, void* H, int M, int N,
                                     int K, int lda, int ldb, int ldc, int ldh, unsigned a_bytes, unsigned b_bytes,
                                     hipStream_t s) {
  if (M <= 0 || N <= 0 || (N % 128) || (K % 64) || ldh < N / 2) return false;
  const long long cspan = ((long long)(M - 1) * ldc + N) * 2;
  const long long hspan = ((long long)(M - 1) * ldh + N / 2) * 2;
  if (cspan >= (1ll << 32) - 16 || hspan >= (1ll << 32) - 16) return false;
  const long long items = (long long)((M + 255) / 256) * ((N + 255) / 256);
  if (items <= 0 || items >= (1ll << 31)) return false;
  const int grid = (int)std::min<long long>(items, g4_cu_count());
  const Rope rope = {nullptr, nullptr, 0, 64};
  const Dual dual = {nullptr, nullptr, 0x7fffffff, lda, ldb, 0u, 0u};
  const SwiOut swo = {(bf16*)H, ldh, (unsigned)hspan};
  gemm4_k<true, true, 0, 0, true, 1, 256, 0, true><<<grid, 256, 0, s>>>(
      (const bf16*)A, (const bf16*)B, C, bias, M, N, K, lda, ldb, ldc, K, 1, 0, a_bytes, b_bytes, (unsigned)cspan, rope,
      g_g4_group_m, dual, 0, nullptr, swo);
  return true;
}

// Down-projection data gradient with the SwiGLU backward in the epilogue (SwiBwd): A = dy
// [M, K] (K-major), B = W_down [K, F] (F contiguous), gu [M, 2F] (interleaved if perm), dgu
// [M, 2F] natural, part [2 * ceil(M / 256), 2F] fp32 (every row written).  Returns false
// (nothing launched) where the 256-wide FAST kernel does not apply.
// gate / up row blocks in flight in the SWB epilogue (1 or 2; A/B hook, tools/ab_attr.py)
static int g_g4_swb_depth = 2;
extern "C" void dpfs_gemm4_swb_depth(int d) { g_g4_swb_depth = d == 1 ? 1 : 2; }

extern "C" bool dpfs_gemm4_nn_swiglu_bwd(const void* A, const void* B, const void* gu, void* dgu, float* part, int M,
                                         int F, int K, int lda, int ldb, int ldgu, int lddgu, int perm,
                                         unsigned a_bytes, unsigned b_bytes, hipStream_t s) {
  if (M <= 0 || F <= 0 || (F % 64) || (K % 64) || lda % 8 || ldb % 8 || ldgu % 8 || lddgu % 8) return false;
  if (ldgu < 2 * F || lddgu < 2 * F) return false;
  const long long guspan = ((long long)(M - 1) * ldgu + 2 * F) * 2;
  const long long dspan = ((long long)(M - 1) * lddgu + 2 * F) * 2;
  const long long tiles_m = (M + 255) / 256;
  const long long pspan = tiles_m * 2 * 2LL * F * 4;
  if (guspan >= (1ll << 32) - 16 || dspan >= (1ll << 32) - 16 || pspan >= (1ll << 32) - 16) return false;
  const long long items = tiles_m * ((F + 255) / 256);
  if (items <= 0 || items >= (1ll << 31)) return false;
  const int grid = (int)std::min<long long>(items, g4_cu_count());
  const Rope rope = {nullptr, nullptr, 0, 64};
  const Dual dual = {nullptr, nullptr, 0x7fffffff, lda, ldb, 0u, 0u};
  // no partials buffer (no bias gradient): a zero-record descriptor drops every partial store
  const SwiBwd swb = {(const bf16*)gu, (bf16*)dgu, part, ldgu, lddgu, perm ? 1 : 0, (unsigned)guspan, (unsigned)dspan,
                      part ? (unsigned)pspan : 0u};
  if (g_g4_swb_depth == 1)
    gemm4_k<true, false, 0, 0, true, 1, 256, 0, false, 1><<<grid, 256, 0, s>>>(
        (const bf16*)A, (const bf16*)B, nullptr, nullptr, M, F, K, lda, ldb, F, K, 1, 0, a_bytes, b_bytes, 0u, rope,
        g_g4_group_m, dual, 0, nullptr, SwiOut{}, swb);
  else
    gemm4_k<true, false, 0, 0, true, 1, 256, 0, false, 2><<<grid, 256, 0, s>>>(
        (const bf16*)A, (const bf16*)B, nullptr, nullptr, M, F, K, lda, ldb, F, K, 1, 0, a_bytes, b_bytes, 0u, rope,
        g_g4_group_m, dual, 0, nullptr, SwiOut{}, swb);
  return true;
}

// Stream-K (gemm4_k's SK) applicability and workspace: plain bf16 NT / NN whose 256 x 256
// tiles number exactly 1.5 per CU, K a multiple of 128.  Floats of workspace (partials, flags,
// error word), -1 where it does not apply.
extern "C" long long dpfs_gemm4_sk_ws(int M, int N, int K) {
  const int cus = g4_cu_count();
  if (M <= 0 || N <= 0 || K <= 0 || cus % 2 || K % 128) return -1;
  const long long tiles = (long long)((M + 255) / 256) * ((N + 255) / 256);
  if (tiles * 2 != 3LL * cus) return -1;
  const long long E = cus / 2;
  return E * 4 * 16384 + E * 4 + 4;
}
static float* g_g4_sk_ws = nullptr;
static long long g_g4_sk_ws_floats = 0;
extern "C" void dpfs_gemm4_set_sk_ws(float* p, long long n) {
  g_g4_sk_ws = p;
  g_g4_sk_ws_floats = n;
}
// Sticky error word of the stream-K hand-off: host-mapped (the host reads it without a device
// sync) and never cleared by a launch, so a consumer whose bounded wait for its producer's
// partial timed out (its tile is then wrong) is reported by the next dpfs_gemm4_sk_error()
// (ops.check_device_errors(), called by the engines after every step) instead of passing
// silently.  Allocated on the first stream-K launch.
static unsigned* g_g4_sk_err_host = nullptr;
static unsigned* g_g4_sk_err_dev = nullptr;
static unsigned* sk_err_word() {
  if (!g_g4_sk_err_dev) {
    unsigned* p = nullptr;
    if (hipHostMalloc((void**)&p, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return nullptr;
    *p = 0u;
    unsigned* d = nullptr;
    if (hipHostGetDevicePointer((void**)&d, p, 0) != hipSuccess) {
      hipHostFree(p);
      return nullptr;
    }
    g_g4_sk_err_host = p;
    g_g4_sk_err_dev = d;
  }
  return g_g4_sk_err_dev;
}
extern "C" int dpfs_gemm4_sk_error(int reset) {
  if (!g_g4_sk_err_host) return 0;
  const int v = (int)__atomic_load_n(g_g4_sk_err_host, __ATOMIC_RELAXED);
  if (reset) __atomic_store_n(g_g4_sk_err_host, 0u, __ATOMIC_RELAXED);
  return v;
}
// Test hook: the next stream-K launch runs its consumers with their producers' flags never
// set (the producers skip the flag store), so every consumer's wait times out.
static int g_g4_sk_starve = 0;
extern "C" void dpfs_gemm4_sk_starve(int on) { g_g4_sk_starve = on; }

// Launch v4.  layout: 0 = NT (A K-major, B K-major), 1 = NN (B MN-major), 2 = TN (both
// MN-major, fp32 out).  Returns false (nothing launched) when a span does not fit the 32-bit
// buffer descriptors or a contiguous dimension is not a multiple of 8.
extern "C" bool dpfs_gemm4_launch(int layout, int out_f32, const void* A, const void* B, void* C, const float* bias,
                                  int M, int N, int K, int lda, int ldb, int ldc, int kps, int splits,
                                  long long slab_stride, unsigned a_bytes, unsigned b_bytes, const int64_t* rope_pos,
                                  const float* rope_tab, int rope_cols, int rope_hd, const void* A2, const void* B2,
                                  int k_switch, int lda2, int ldb2, unsigned a2_bytes, unsigned b2_bytes,
                                  int bn_force, hipStream_t s) {
  // bn_force: tile width of a non-split bf16 GEMM, 0 = chosen per shape, 256 / 192 forced;
  // | 0x100: the bf16 output written with non-temporal stores (plain NT / NN); | 0x200: the
  // stream-K kernel where it applies (dpfs_gemm4_sk_ws, workspace set by dpfs_gemm4_set_sk_ws)
  const bool ntst = (bn_force & 0x100) != 0;
  const bool skreq = (bn_force & 0x200) != 0;
  bn_force &= 0xff;
  if (M <= 0 || N <= 0 || (N % 8) || (K % 8)) return false;
  if (layout == 2 && (M % 8)) return false;
  if (rope_cols > 0 && rope_hd != 64 && rope_hd != 128) return false;
  if (kps % 32) return false;
  const long long cspan = ((long long)(M - 1) * ldc + N) * (out_f32 ? 4 : 2);
  if (cspan >= (1ll << 32) - 16) return false;
  // 256 x 192 tiles where whole waves of tiles over the CUs come out shorter: 384 tiles of
  // 256 x 256 (N = 768 at 32k rows) are 1.5 per CU, i.e. two rounds on half the chip; 512
  // tiles of 256 x 192 are two full rounds of 3/4 the work.  Priced at 0.8 of a 256-wide
  // tile (its 7 DMA pieces per 48 MFMAs vs 8 per 64).
  const int cus = g4_cu_count();
  int bn = 256;
  if (!out_f32 && splits == 1 && rope_cols == 0) {
    if (bn_force == 192) {
      bn = 192;
    } else if (bn_force == 0) {
      const long long tm = (M + 255) / 256;
      const long long r256 = (tm * ((N + 255) / 256) + cus - 1) / cus;
      const long long r192 = (tm * ((N + 191) / 192) + cus - 1) / cus;
      if (r192 * 0.8 < r256 * 0.95) bn = 192;
    }
  }
  const long long items = (long long)((M + 255) / 256) * ((N + bn - 1) / bn) * splits;
  if (items <= 0 || items >= (1ll << 31)) return false;
  const int grid = (int)std::min<long long>(items, cus);
  const Rope rope = {rope_pos, rope_tab, rope_cols, rope_hd};
  const Dual dual = {(const bf16*)A2, (const bf16*)B2, A2 ? k_switch : 0x7fffffff, lda2, ldb2, a2_bytes, b2_bytes};
  const unsigned cb = (g_g4_ablate & 1) ? 0u : (unsigned)cspan;
  if (g_g4_ablate & 2) {
    a_bytes = b_bytes = a2_bytes = b2_bytes = 0u;
  }
  // FAST (descriptor-advancing DMA stream): every item's K range a multiple of 64
  // (not under the zero-operand ablation: FAST's per-item record counts are the bytes past the
  // item's K offset, which a zero-record descriptor would underflow)
  const bool fast = g_g4_sched != 2 && !(g_g4_ablate & 2) && K % 64 == 0 && kps % 64 == 0 &&
                    (!A2 || k_switch % 64 == 0);
  const int sched = g_g4_sched == 1 ? 0 : 1;
#define G4_ARGS                                                                                            \
  (const bf16*)A, (const bf16*)B, C, bias, M, N, K, lda, ldb, ldc, kps, splits, slab_stride, a_bytes, b_bytes, cb, \
      rope, g_g4_group_m, dual, g_g4_ablate & ~3, nullptr
#define G4_LAUNCH(AK_, BK_, OUT_)                                                                    \
  do {                                                                                            \
    if constexpr (AK_ && BK_ && OUT_ == 0) {                                                      \
      if (rope_cols > 0) {                                                                        \
        if (fast && rope_hd == 64)                                                                \
          gemm4_k<AK_, BK_, OUT_, 0, true, 1, 256, 64><<<grid, 256, 0, s>>>(G4_ARGS);        \
        else if (fast)                                                                            \
          gemm4_k<AK_, BK_, OUT_, 0, true, 1, 256, 128><<<grid, 256, 0, s>>>(G4_ARGS);       \
        else if (rope_hd == 64)                                                                   \
          gemm4_k<AK_, BK_, OUT_, 0, false, 0, 256, 64><<<grid, 256, 0, s>>>(G4_ARGS);       \
        else                                                                                      \
          gemm4_k<AK_, BK_, OUT_, 0, false, 0, 256, 128><<<grid, 256, 0, s>>>(G4_ARGS);      \
        break;                                                                                    \
      }                                                                                           \
    }                                                                                             \
    if constexpr (!AK_ && !BK_ && OUT_ == 1) {                                                    \
      if (fast && sched == 1 && g_g4_m32) {                                                       \
        if (g_g4_br_tn == 1)                                                                      \
          gemm4_k<false, false, 1, 0, true, 1, 256, 0, false, false, 1, 0, true>                  \
              <<<grid, 256, 0, s>>>(G4_ARGS);                                                     \
        else if (g_g4_br_tn == 2)                                                                 \
          gemm4_k<false, false, 1, 0, true, 1, 256, 0, false, false, 2, 0, true>                  \
              <<<grid, 256, 0, s>>>(G4_ARGS);                                                     \
        else                                                                                      \
          gemm4_k<false, false, 1, 0, true, 1, 256, 0, false, false, 0, 0, true>                  \
              <<<grid, 256, 0, s>>>(G4_ARGS);                                                     \
        break;                                                                                    \
      }                                                                                           \
    }                                                                                             \
    if constexpr (AK_ && OUT_ == 1) {                                                             \
      if (fast && sched == 1 && (g_g4_m32k & 1)) {                                                \
        gemm4_k<AK_, BK_, 1, 0, true, 1, 256, 0, false, false, 0, 0, true>                        \
            <<<grid, 256, 0, s>>>(G4_ARGS);                                                       \
        break;                                                                                    \
      }                                                                                           \
    }                                                                                             \
    if constexpr (AK_ && OUT_ == 0) {                                                             \
      if (fast && sched == 1 && (g_g4_m32k & 2) && bn == 256 && rope_cols == 0) {                 \
        if (ntst)                                                                                 \
          gemm4_k<AK_, BK_, 0, 0, true, 1, 256, 0, false, false, 0, 2, true>                      \
              <<<grid, 256, 0, s>>>(G4_ARGS);                                                     \
        else                                                                                      \
          gemm4_k<AK_, BK_, 0, 0, true, 1, 256, 0, false, false, 0, 0, true>                      \
              <<<grid, 256, 0, s>>>(G4_ARGS);                                                     \
        break;                                                                                    \
      }                                                                                           \
    }                                                                                             \
    if (fast && sched == 1 && OUT_ == 0 && ntst && rope_cols == 0) {                             \
      if (bn == 192)                                                                              \
        gemm4_k<AK_, BK_, OUT_, 0, true, 1, 192, 0, false, false, 0, 2><<<grid, 256, 0, s>>>(G4_ARGS); \
      else                                                                                        \
        gemm4_k<AK_, BK_, OUT_, 0, true, 1, 256, 0, false, false, 0, 2><<<grid, 256, 0, s>>>(G4_ARGS); \
    } else if (fast && sched == 1) {                                                              \
      if (OUT_ == 0 && bn == 192) {                                                               \
        if (g_g4_br == 1)                                                                         \
          gemm4_k<AK_, BK_, OUT_, 0, true, 1, (OUT_ == 0 ? 192 : 256), 0, false, false, 1>         \
              <<<grid, 256, 0, s>>>(G4_ARGS);                                                     \
        else if (g_g4_br == 2)                                                                    \
          gemm4_k<AK_, BK_, OUT_, 0, true, 1, (OUT_ == 0 ? 192 : 256), 0, false, false, 2>         \
              <<<grid, 256, 0, s>>>(G4_ARGS);                                                     \
        else                                                                                      \
          gemm4_k<AK_, BK_, OUT_, 0, true, 1, (OUT_ == 0 ? 192 : 256)><<<grid, 256, 0, s>>>(G4_ARGS); \
      } else if (g_g4_br == 1) {                                                                  \
        gemm4_k<AK_, BK_, OUT_, 0, true, 1, 256, 0, false, false, 1><<<grid, 256, 0, s>>>(G4_ARGS); \
      } else if (g_g4_br == 2) {                                                                  \
        gemm4_k<AK_, BK_, OUT_, 0, true, 1, 256, 0, false, false, 2><<<grid, 256, 0, s>>>(G4_ARGS); \
      } else {                                                                                    \
        gemm4_k<AK_, BK_, OUT_, 0, true, 1><<<grid, 256, 0, s>>>(G4_ARGS);                   \
      }                                                                                           \
    } else if (fast) {                                                                            \
      if (OUT_ == 0 && bn == 192)                                                                 \
        gemm4_k<AK_, BK_, OUT_, 0, true, 0, (OUT_ == 0 ? 192 : 256)><<<grid, 256, 0, s>>>(G4_ARGS); \
      else                                                                                        \
        gemm4_k<AK_, BK_, OUT_, 0, true, 0><<<grid, 256, 0, s>>>(G4_ARGS);                   \
    } else if (OUT_ == 0 && bn == 192) {                                                          \
      gemm4_k<AK_, BK_, OUT_, 0, false, 0, (OUT_ == 0 ? 192 : 256)><<<grid, 256, 0, s>>>(G4_ARGS); \
    } else {                                                                                      \
      gemm4_k<AK_, BK_, OUT_><<<grid, 256, 0, s>>>(G4_ARGS);                                 \
    }                                                                                             \
  } while (0)
  if (skreq && layout != 2 && !out_f32 && splits == 1 && rope_cols == 0 && fast && sched == 1 && !A2 && !g_g4_ablate) {
    const long long need = dpfs_gemm4_sk_ws(M, N, K);
    if (need > 0 && g_g4_sk_ws && g_g4_sk_ws_floats >= need) {
      const int E = cus / 2;
      SkArgs sk;
      sk.part = g_g4_sk_ws;
      sk.flags = reinterpret_cast<unsigned*>(g_g4_sk_ws + (long long)E * 4 * 16384);
      sk.err = sk_err_word();
      if (!sk.err) return false;
      sk.extra = E;
      sk.starve = g_g4_sk_starve;
      g_g4_sk_starve = 0;
      if (hipMemsetAsync(sk.flags, 0, (size_t)(E * 4 + 1) * 4, s) != hipSuccess) return false;
#define G4_SK(AK_, BK_, SA_)                                                                                  \
  gemm4_k<AK_, BK_, 0, 0, true, 1, 256, 0, false, 0, 0, SA_, false, false, true><<<cus, 256, 0, s>>>(       \
      (const bf16*)A, (const bf16*)B, C, bias, M, N, K, lda, ldb, ldc, K, 1, 0, a_bytes, b_bytes, cb, rope, \
      g_g4_group_m, dual, 0, nullptr, SwiOut{}, SwiBwd{}, TnGroup{}, sk)
      if (layout == 0) {
        if (ntst) G4_SK(true, true, 2);
        else G4_SK(true, true, 0);
      } else {
        if (ntst) G4_SK(true, false, 2);
        else G4_SK(true, false, 0);
      }
#undef G4_SK
      return true;
    }
  }
  if ((g_g4_ablate & 32) && g_g4_diag && layout == 0 && !out_f32 && bn == 256) {
    gemm4_k<true, true, 0, 2, true, 1><<<grid, 256, 0, s>>>((const bf16*)A, (const bf16*)B, C, bias, M, N, K, lda,
                                                            ldb, ldc, kps, splits, slab_stride, a_bytes, b_bytes, cb,
                                                            rope, g_g4_group_m, dual, g_g4_ablate & ~51, g_g4_diag);
    return true;
  }
  if ((g_g4_ablate & (4 | 8 | 1024)) && layout == 0 && !out_f32 && bn == 256 && fast && rope_cols == 0) {
    // the ablation build (1024: the same build with no ablation, the cost of its branches)
    gemm4_k<true, true, 0, 3, true, 1><<<grid, 256, 0, s>>>((const bf16*)A, (const bf16*)B, C, bias, M, N, K, lda,
                                                            ldb, ldc, kps, splits, slab_stride, a_bytes, b_bytes, cb,
                                                            rope, g_g4_group_m, dual, g_g4_ablate, nullptr);
    return true;
  }
  if ((g_g4_ablate & 128) && layout == 0 && !out_f32 && bn == 256 && fast && rope_cols == 0) {
    // A/B: the bf16 epilogue stores with the non-temporal hint (streaming output, aux nt)
    gemm4_k<true, true, 0, 0, true, 1, 256, 0, false, false, 0, 2><<<grid, 256, 0, s>>>(
        (const bf16*)A, (const bf16*)B, C, bias, M, N, K, lda, ldb, ldc, kps, splits, slab_stride, a_bytes, b_bytes, cb,
        rope, g_g4_group_m, dual, 0, nullptr);
    return true;
  }
  if ((g_g4_ablate & (16 | 32)) && g_g4_diag && layout == 2 && fast && g_g4_m32) {
    // TN 32x32x16: the DIAG builds (16: per-wave cycle split; 32: the same with no DMA issued)
    const Rope rp = rope;
    if (g_g4_ablate & 32)
      gemm4_k<false, false, 1, 2, true, 1, 256, 0, false, false, 0, 0, true><<<grid, 256, 0, s>>>(
          (const bf16*)A, (const bf16*)B, C, bias, M, N, K, lda, ldb, ldc, kps, splits, slab_stride, a_bytes, b_bytes,
          cb, rp, g_g4_group_m, dual, 0, g_g4_diag);
    else
      gemm4_k<false, false, 1, 1, true, 1, 256, 0, false, false, 0, 0, true><<<grid, 256, 0, s>>>(
          (const bf16*)A, (const bf16*)B, C, bias, M, N, K, lda, ldb, ldc, kps, splits, slab_stride, a_bytes, b_bytes,
          cb, rp, g_g4_group_m, dual, 0, g_g4_diag);
    return true;
  }
  if ((g_g4_ablate & 16) && g_g4_diag && layout == 0 && !out_f32 && bn == 256 && fast) {
    gemm4_k<true, true, 0, 1, true, 1><<<grid, 256, 0, s>>>((const bf16*)A, (const bf16*)B, C, bias, M, N, K, lda,
                                                            ldb, ldc, kps, splits, slab_stride, a_bytes, b_bytes, cb,
                                                            rope, g_g4_group_m, dual, g_g4_ablate & ~19, g_g4_diag);
    return true;
  }
  if (layout == 0) {
    if (out_f32) G4_LAUNCH(true, true, 1);
    else G4_LAUNCH(true, true, 0);
  } else if (layout == 1) {
    if (out_f32) G4_LAUNCH(true, false, 1);
    else G4_LAUNCH(true, false, 0);
  } else {
    if (!out_f32) return false;
    G4_LAUNCH(false, false, 1);
  }
#undef G4_ARGS
#undef G4_LAUNCH
  return true;
}

// ---------------------------------------------------------------- grouped weight gradients --
// C_g (+)= A_g^T B_g for up to 4 TN GEMMs over the same K (a layer's weight gradients: A_g
// [K, M_g], B_g [K, N_g], MN-contiguous), as ONE persistent 32x32x16 launch plus at most one
// reduction launch: every GEMM takes the same K-split length, chosen for the group's total
// tile count (a makespan model as tn_v2_splits: rounds of the CUs x split length, plus the
// slabs' write + read), so all items are equally long and the rounds fill the chip; the
// separate launches each paid a ramp / tail and one slab round trip per GEMM.
static int tn_group_splits(int n, const int* M, const int* N, int K, long long* mn_out) {
  long long tiles = 0, mn = 0;
  for (int g = 0; g < n; ++g) {
    tiles += (long long)((M[g] + 255) / 256) * ((N[g] + 255) / 256);
    mn += (long long)M[g] * N[g];
  }
  *mn_out = mn;
  const int cus = g4_cu_count();
  int best = 1;
  double best_t = 1e300;
  for (int S = 1; S <= 64; ++S) {
    if (S > 1 && K / S < 512) break;
    const long long kps = ((K + S - 1) / S + 63) / 64;
    const long long se = (K + kps * 64 - 1) / (kps * 64);
    if (se != S) continue;   // (S and S - 1 giving the same split length)
    const long long rounds = (tiles * S + cus - 1) / cus;
    const double t = (double)rounds * kps * 1.95 + (S > 1 ? (double)S * mn * 8.0 / 4.0e6 : 0.0);
    if (t < best_t * 0.97) {
      best_t = t;
      best = S;
    }
  }
  return best;
}

// The group's K-split plan: S splits of kps rows (a multiple of 64) over K = K0 + K1 rows.
// With a second buffer (K1 > 0) each buffer is split on its own -- S0 splits over K0 and S1
// over K1 with one kps -- and the kernel sees K0 padded to S0 kps (*kswitch): no work item
// straddles the buffers, and the padding rows past K0 read zeros (past the first buffers'
// descriptors).  S0 / S1 by the same makespan model as tn_group_splits.
static bool tn_group_plan(int n, const int* M, const int* N, int K0, int K1, int* S_out, int* kps_out, long long* mn,
                          int* kswitch) {
  const int K = K0 + K1;
  int S = tn_group_splits(n, M, N, K, mn);
  int kps = ((K + S - 1) / S + 63) / 64 * 64;
  *kswitch = 0x7fffffff;
  if (K1 > 0) {
    if (K0 % 64 || K1 % 64) return false;
    long long tiles = 0;
    for (int g = 0; g < n; ++g) tiles += (long long)((M[g] + 255) / 256) * ((N[g] + 255) / 256);
    const int cus = g4_cu_count();
    double best_t = 1e300;
    int bS = 0, bk = 0, bs0 = 0;
    for (int S0 = 1; S0 <= 32; ++S0) {
      const int S1 = std::max(1, (int)((double)S0 * K1 / K0 + 0.5));
      const int k0 = ((K0 + S0 - 1) / S0 + 63) / 64 * 64, k1 = ((K1 + S1 - 1) / S1 + 63) / 64 * 64;
      const int kp = std::max(k0, k1);
      if (S0 + S1 > 2 && kp < 512) break;
      const int s0 = (K0 + kp - 1) / kp, s1 = (K1 + kp - 1) / kp;
      const long long rounds = (tiles * (s0 + s1) + cus - 1) / cus;
      const double t = (double)rounds * kp * 1.95 + (double)(s0 + s1) * (*mn) * 8.0 / 4.0e6;
      if (t < best_t * 0.97) {
        best_t = t;
        bS = s0 + s1;
        bk = kp;
        bs0 = s0;
      }
    }
    if (bS <= 0) return false;
    S = bS;
    kps = bk;
    *kswitch = bs0 * bk;
  }
  *S_out = S;
  *kps_out = kps;
  return true;
}

// Floats of slab workspace dpfs_gemm_tn_group needs (0: none).  -1: the group does not run
// grouped (K % 64, unaligned dims, spans past the 32-bit descriptors, the 16x16x32 TN form).
// K1 > 0: the rows continue in second buffers (lda2 / ldb2) for K1 more rows.
extern "C" long long dpfs_gemm_tn_group_ws(int n, const int* M, const int* N, const int* lda, const int* ldb, int K,
                                           const int* acc, const int* lda2, const int* ldb2, int K1) {
  if (n < 1 || n > 4 || K % 64 || !g_g4_m32 || K <= 0 || K1 < 0 || (K1 && (K1 % 64 || !lda2 || !ldb2))) return -1;
  bool any_acc = false;
  for (int g = 0; g < n; ++g) {
    if (M[g] <= 0 || N[g] <= 0 || M[g] % 8 || N[g] % 8 || lda[g] < M[g] || ldb[g] < N[g]) return -1;
    if (((long long)(K - 1) * lda[g] + M[g]) * 2 >= (1ll << 32) - 16) return -1;
    if (((long long)(K - 1) * ldb[g] + N[g]) * 2 >= (1ll << 32) - 16) return -1;
    if (K1) {
      if (lda2[g] < M[g] || ldb2[g] < N[g] || lda2[g] % 8 || ldb2[g] % 8) return -1;
      if (((long long)(K1 - 1) * lda2[g] + M[g]) * 2 >= (1ll << 32) - 16) return -1;
      if (((long long)(K1 - 1) * ldb2[g] + N[g]) * 2 >= (1ll << 32) - 16) return -1;
    }
    if ((long long)M[g] * N[g] * 4 >= (1ll << 32) - 16) return -1;
    any_acc |= acc[g] != 0;
  }
  long long mn;
  int S, kps, ksw;
  if (!tn_group_plan(n, M, N, K, K1, &S, &kps, &mn, &ksw)) return -1;
  return (S > 1 || any_acc) ? (long long)S * mn : 0;
}

extern "C" int dpfs_gemm_tn_group(int n, const void* const* A, const void* const* B, float* const* C, const int* M,
                                  const int* N, const int* lda, const int* ldb, const int* acc, int K, float* ws,
                                  long long ws_floats, const void* const* A2, const void* const* B2, const int* lda2,
                                  const int* ldb2, int K1, hipStream_t s) {
  const long long need = dpfs_gemm_tn_group_ws(n, M, N, lda, ldb, K, acc, lda2, ldb2, K1);
  if (need < 0 || (need > 0 && (ws == nullptr || ws_floats < need))) return 0;
  long long mn;
  int S, kps, ksw;
  if (!tn_group_plan(n, M, N, K, K1, &S, &kps, &mn, &ksw)) return 0;
  const bool slabs = need > 0;
  TnGroup grp{};
  grp.n = n;
  grp.k_switch = ksw;   // (K1 > 0: K0 padded to whole splits; else none)
  grp.k0 = K1 ? K : 0x7fffffff;
  RedGroup red{};
  red.n = n;
  red.S = S;
  long long items = 0, off = 0;
  for (int g = 0; g < n; ++g) {
    TnGemm& d = grp.d[g];
    d.A = (const bf16*)A[g];
    d.B = (const bf16*)B[g];
    d.M = M[g];
    d.N = N[g];
    d.lda = lda[g];
    d.ldb = ldb[g];
    d.ldc = N[g];
    d.tiles_m = (M[g] + 255) / 256;
    d.tiles_n = (N[g] + 255) / 256;
    d.item0 = (int)items;
    d.a_bytes = (unsigned)(((long long)(K - 1) * lda[g] + M[g]) * 2);
    d.b_bytes = (unsigned)(((long long)(K - 1) * ldb[g] + N[g]) * 2);
    d.c_bytes = (unsigned)((long long)M[g] * N[g] * 4);
    if (K1) {
      d.A2 = (const bf16*)A2[g];
      d.B2 = (const bf16*)B2[g];
      d.lda2 = lda2[g];
      d.ldb2 = ldb2[g];
      d.a2_bytes = (unsigned)(((long long)(K1 - 1) * lda2[g] + M[g]) * 2);
      d.b2_bytes = (unsigned)(((long long)(K1 - 1) * ldb2[g] + N[g]) * 2);
    }
    const long long ng = (long long)M[g] * N[g];
    d.C = slabs ? ws + off : C[g];
    d.slab_stride = slabs ? ng : 0;
    red.pre[g] = off / S;
    red.ws[g] = ws + off;
    red.out[g] = C[g];
    red.acc[g] = acc[g];
    if (slabs) off += S * ng;
    items += (long long)d.tiles_m * d.tiles_n * S;
  }
  red.pre[n] = mn;
  if (items >= (1ll << 31)) return 0;
  grp.total = (int)items;
  const int grid = (int)std::min<long long>(items, g4_cu_count());
  const Rope rope = {nullptr, nullptr, 0, 64};
  const Dual dual = {nullptr, nullptr, 0x7fffffff, 0, 0, 0u, 0u};
#define G4_GRP(BR_)                                                                                         \
  gemm4_k<false, false, 1, 0, true, 1, 256, 0, false, false, BR_, 0, true, true><<<grid, 256, 0, s>>>(       \
      grp.d[0].A, grp.d[0].B, grp.d[0].C, nullptr, 256, 256, K1 ? ksw + K1 : K, lda[0], ldb[0], N[0], kps, S, 0, \
      grp.d[0].a_bytes, grp.d[0].b_bytes, grp.d[0].c_bytes, rope, g_g4_group_m, dual, 0, nullptr, SwiOut{},     \
      SwiBwd{}, grp)
  if (g_g4_br_tn == 1) G4_GRP(1);
  else if (g_g4_br_tn == 2) G4_GRP(2);
  else G4_GRP(0);
#undef G4_GRP
  if (slabs) {
    long long gr = (mn / 4 + 255) / 256;
    if (gr > 4096) gr = 4096;
    splitk_reduce_group_k<<<(int)gr, 256, 0, s>>>(red);
  }
  return 1;
}
