// Helpers shared by the attention kernels (attention.hip: forward, the dQ + dK/dV backward
// pair, decode-independent; attention_fused.hip: the fused head_dim-64 backward): LDS
// swizzles, asm transposed reads / single-issue f32 ops, the 32x32x16 MFMA macro, the Q / dO
// LDS-DMA stage, the whole-row epilogue staging and the QKV bias-gradient reduction.
#pragma once

#include "common.h"

namespace dpfs {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

typedef short s16x8 __attribute__((ext_vector_type(8)));

// Swizzled byte offset of 16-byte chunk `ch` of row `r` in a [rows][HD] bf16 tile.
template <int HD>
__device__ __forceinline__ int sw_off(int r, int ch) {
  constexpr int RB = HD * 2;
  int f;
  if (HD == 32) f = ((r >> 2) & 1) << 1;
  else if (HD == 64) f = ((r >> 1) & 3) << 1;
  else f = (r & 7) << 1;
  return r * RB + ((ch ^ f) << 4);
}

// Row read: lane holds X[rb + (l&15)][kb + 8(l>>4) + j]  (16x16x32 A/B operand, K-contiguous).
template <int HD>
__device__ __forceinline__ bf16x8 row_frag(const char* lds, int rb, int kb) {
  const int l = lane_id();
  return *reinterpret_cast<const bf16x8*>(lds + sw_off<HD>(rb + (l & 15), (kb >> 3) + (l >> 4)));
}

// Transposed read with the permuted k-slots used for P^T / dS^T operands:
// lane l (g = l>>4) gets X[r0 + 4g + j][c0 + (l&15)] for j<4 and X[r0 + 16 + 4g + j-4][...] for j>=4.
template <int HD>
__device__ __forceinline__ bf16x8 tr_frag(const char* lds, int r0, int c0) {
  const int l = lane_id();
  const int i = l & 15, q = i >> 2, p = i & 3, g = l >> 4;
  const int col = c0 + 4 * p;
  const int ch = col >> 3;
  const int r_lo = r0 + 4 * g + q;
  const int r_hi = r_lo + 16;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(lds + sw_off<HD>(r_lo, ch) + (p & 1) * 8));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(lds + sw_off<HD>(r_hi, ch) + (p & 1) * 8));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// tr_frag through inline asm.  hipcc puts an `s_waitcnt vmcnt(0)` in front of the
// ds_read_b64_tr_b16 builtin whenever any LDS-DMA is in flight (it cannot tell the DMA's LDS
// destination from the read's), which drains a prefetch ring.  The asm form is invisible to
// its bookkeeping: the caller retires the reads with tr_wait (one `s_waitcnt lgkmcnt(0)`
// statement naming every destination "+v", guide §5.7 item 1 form (ii)) before any use,
// and orders the LDS-DMA data with its own vmcnt + barrier.  EXEC must be all ones.
__device__ __forceinline__ unsigned lds_u32(const char* p) {
  return (unsigned)(size_t)((__attribute__((address_space(3))) const char*)p);
}
// Scalar f32 add / multiply as single instructions: beside MFMAs a v_pk_*_f32 costs more issue
// time than the two scalar ops it replaces (MI355X_MICROARCH constants), and hipcc SLP-packs
// adjacent scalar adds / multiplies into them under -O3.
__device__ __forceinline__ float vaddf(float a, float b) {
  float r;
  asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vmulf(float a, float b) {
  float r;
  asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// max of finite / -inf values as single instructions (no canonicalisation)
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float vmax2(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ s16x4 ds_tr16(const char* p) {
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(lds_u32(p)));
  return r;
}
// ... at a byte offset in the instruction's offset field: one address per row group instead of
// one v_add per read.  `off` is a constant after unrolling (the switch folds away); the
// offsets of the tiles' row steps (16 or 8 rows of 128 / 256 B) have cases, any other adds.
template <int OFF>
__device__ __forceinline__ s16x4 ds_tr16_at(const char* p) {
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(lds_u32(p)), "n"(OFF));
  return r;
}
__device__ __forceinline__ s16x4 ds_tr16_off(const char* p, int off) {
  switch (off) {
#define ATT_TR(O) \
  case O: return ds_tr16_at<O>(p);
    ATT_TR(0) ATT_TR(1024) ATT_TR(2048) ATT_TR(3072) ATT_TR(4096) ATT_TR(5120) ATT_TR(6144) ATT_TR(7168)
    ATT_TR(8192) ATT_TR(10240) ATT_TR(12288) ATT_TR(14336) ATT_TR(16384) ATT_TR(18432) ATT_TR(20480)
    ATT_TR(22528) ATT_TR(24576) ATT_TR(26624) ATT_TR(28672) ATT_TR(30720)
#undef ATT_TR
    default: return ds_tr16(p + off);
  }
}
template <int HD>
__device__ __forceinline__ void tr_frag_asm(const char* lds, int r0, int c0, s16x4& lo, s16x4& hi) {
  const int l = lane_id();
  const int i = l & 15, q = i >> 2, p = i & 3, g = l >> 4;
  const int col = c0 + 4 * p;
  const int ch = col >> 3;
  const int r_lo = r0 + 4 * g + q;
  lo = ds_tr16(lds + sw_off<HD>(r_lo, ch) + (p & 1) * 8);
  hi = ds_tr16(lds + sw_off<HD>(r_lo + 16, ch) + (p & 1) * 8);
}
__device__ __forceinline__ bf16x8 tr_join(const s16x4& lo, const s16x4& hi) {
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
// Retire every outstanding LDS read and pin the 8 fragments (16 halves) behind the wait.
__device__ __forceinline__ void tr_wait8(s16x4 (&x)[16]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
                 "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]),
                 "+v"(x[15]));
}

// Pack two 16x16 C tiles (rows 4g+j of tile a, of tile b) into the permuted 8-slot operand.
__device__ __forceinline__ bf16x8 pack_pt(const f32x4& a, const f32x4& b) {
  bf16x8 r;
  r[0] = (bf16)a[0]; r[1] = (bf16)a[1]; r[2] = (bf16)a[2]; r[3] = (bf16)a[3];
  r[4] = (bf16)b[0]; r[5] = (bf16)b[1]; r[6] = (bf16)b[2]; r[7] = (bf16)b[3];
  return r;
}

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

// Max / sum over the four 16-lane groups of a wave (lanes l, l^16, l^32, l^48) with the
// CDNA4 half-exchange permlanes (VALU) instead of ds_bpermute round trips through the LDS
// unit: v_permlane16_swap with vdst = src = x leaves {x from my group, x from group ^1} in
// the two results, v_permlane32_swap likewise for group ^2.
__device__ __forceinline__ float group4_max(float x) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float group4_sum(float x) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}


typedef float f32x2v __attribute__((ext_vector_type(2)));   // a register pair (v_pk_*_f32)
#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)

// max / sum of x over lanes l and l ^ 32 (the two lanes of one 32x32 C/D column).
__device__ __forceinline__ float pair_max(float x) {
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float pair_sum(float x) {
  auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}


// s_waitcnt vmcnt(n) for a wave-uniform runtime n (jump over the immediates 0..63).
__device__ __forceinline__ void wait_vm_rt(int n) {
  switch (n) {
#define ATT_W(N_) \
  case N_: wait_vmcnt<N_>(); break;
    ATT_W(0) ATT_W(1) ATT_W(2) ATT_W(3) ATT_W(4) ATT_W(5) ATT_W(6) ATT_W(7) ATT_W(8) ATT_W(9)
    ATT_W(10) ATT_W(11) ATT_W(12) ATT_W(13) ATT_W(14) ATT_W(15) ATT_W(16) ATT_W(17) ATT_W(18)
    ATT_W(19) ATT_W(20) ATT_W(21) ATT_W(22) ATT_W(23) ATT_W(24) ATT_W(25) ATT_W(26) ATT_W(27)
    ATT_W(28) ATT_W(29) ATT_W(30) ATT_W(31) ATT_W(32) ATT_W(33) ATT_W(34) ATT_W(35) ATT_W(36)
    ATT_W(37) ATT_W(38) ATT_W(39) ATT_W(40) ATT_W(41) ATT_W(42) ATT_W(43) ATT_W(44) ATT_W(45)
    ATT_W(46) ATT_W(47) ATT_W(48) ATT_W(49) ATT_W(50) ATT_W(51) ATT_W(52) ATT_W(53) ATT_W(54)
    ATT_W(55) ATT_W(56) ATT_W(57) ATT_W(58) ATT_W(59) ATT_W(60) ATT_W(61) ATT_W(62) ATT_W(63)
#undef ATT_W
    default: wait_vmcnt<0>(); break;
  }
}


template <int HD>
__device__ __forceinline__ int swz_u(int r, int ch) {
  if constexpr (HD == 64) {
    const int m = r >> 1;
    return ch ^ ((m & 7) ^ ((m & 1) << 2));   // hd 64: 8 chunks per row
  } else {
    // hd 128: 16 chunks of 16 B per 256-B row, so every row starts a bank row.  Row reads (16
    // lanes = 16 consecutive rows, one chunk): the XOR term must be a permutation over any 16
    // aligned rows; transposed reads (32 lanes = 4 aligned rows x 4 consecutive chunks of one
    // 64-B span): its bits 2-3 must differ over any 4 aligned rows.  Bit rotation of r & 15
    // does both, and depends on r & 15 only (row + 16 s / + 32 qt stay immediates).
    static_assert(HD == 128, "swz_u: head_dim 64 or 128");
    return ch ^ (((r & 3) << 2) | ((r >> 2) & 3));
  }
}

// Q / dO rows [q0, q0 + 64) and the 64 lse / delta values of a query tile into one stage:
// [Q tile | dO tile | lse (256 B) | delta (256 B) | dummy (512 B)].
// Epilogue of the v3 backward kernels: a wave's 32 x HD accumulator block (lane = row r32,
// registers = columns 32 dt + 8 g + 4 hf + j) goes out as whole rows.  Stored per lane, every
// store instruction touches 32 rows (one 8-byte piece each); staged through the wave's own LDS
// rows (padded: the 32 rows start 16 bytes apart in the banks) each 16-byte read-back covers
// HD / 8 lanes of one row, so a store instruction writes 64 / (HD / 8) whole rows.
template <int HD>
struct RowStage {
  static constexpr int EPR = HD * 2 + 16, BYTES = 32 * EPR, CPR = HD / 8;
  __device__ __forceinline__ static void put(char* ep, const f32x16 (&acc)[HD / 32]) {
    const int l = lane_id(), r32 = l & 31, hf = l >> 5;
#pragma unroll
    for (int dt = 0; dt < HD / 32; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const bf16x4 v = {(bf16)acc[dt][4 * g], (bf16)acc[dt][4 * g + 1], (bf16)acc[dt][4 * g + 2],
                          (bf16)acc[dt][4 * g + 3]};
        *reinterpret_cast<bf16x4*>(ep + r32 * EPR + (32 * dt + 8 * g + 4 * hf) * 2) = v;
      }
  }
  static constexpr int NI = 32 * CPR / 64;   // 16-byte pieces per lane
  // read the wave's rows back, lane l taking pieces 64 i + l (row = piece / CPR): all reads
  // before any store, so no store's data registers are overwritten while it is in flight
  __device__ __forceinline__ static void get(const char* ep, u32x4 (&v)[NI]) {
    const int l = lane_id();
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int idx = 64 * i + l;
      v[i] = *reinterpret_cast<const u32x4*>(ep + (idx / CPR) * EPR + (idx % CPR) * 16);
    }
  }
  // rows row0 + [0, 32) of the T rows at dst (row stride ld elements), by buffer stores: rows
  // >= T fall past the descriptor's record count and are dropped (no branches)
  __device__ __forceinline__ static void put_rows(const u32x4 (&v)[NI], bf16* dst, long long ld, int row0, int T) {
    const int l = lane_id();
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        (void*)dst, (short)0, (int)(((long long)(T - 1) * ld + HD) * 2), 0x00020000);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int idx = 64 * i + l, row = row0 + idx / CPR;
      const unsigned off = row < T ? (unsigned)(((long long)row * ld + (idx % CPR) * 8) * 2) : kOOB;
      __builtin_amdgcn_raw_buffer_store_b128(v[i], r, off, 0, 0);
    }
  }
};

template <int HD>
struct QdoDma3 {
  static constexpr int CPR = HD / 8, TILE = 64 * HD * 2, P = 2 * TILE / 1024, PW = P / 4;
  unsigned voff[PW];
  __device__ __forceinline__ void init(long long ldq, long long lddo) {
    const int l = lane_id(), wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const bool isdo = i >= PW / 2;
      const int jj = wave + 4 * i - (isdo ? P / 2 : 0);
      const int pos = jj * 64 + l;
      const int r = pos / CPR, cp = pos % CPR;
      voff[i] = (unsigned)(((long long)r * (isdo ? lddo : ldq) + swz_u<HD>(r, cp) * 8) * 2);
    }
  }
  __device__ __forceinline__ void issue(const bf16* qb, const bf16* dob, const float* lsb, const float* dlb,
                                        long long ldq, long long lddo, int T, int q0, char* stage) const {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = lane_id();
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(qb + (long long)q0 * ldq), (short)0, (int)(((long long)(T - 1 - q0) * ldq + HD) * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rdo = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(dob + (long long)q0 * lddo), (short)0, (int)(((long long)(T - 1 - q0) * lddo + HD) * 2), 0x00020000);
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const bool isdo = i >= PW / 2;
      const int jj = wave + 4 * i - (isdo ? P / 2 : 0);
      dma16(isdo ? rdo : rq, stage + (isdo ? TILE : 0) + jj * 1024, voff[i]);
    }
    // wave 0: lse, wave 1: delta, waves 2 / 3: a dummy piece (every wave issues PW + 1)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((wave == 1 ? dlb : lsb) + q0), (short)0, (T - q0) * 4, 0x00020000);
    const unsigned soff = wave < 2 ? (unsigned)l * 4u : kOOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(stage + 2 * TILE + wave * 256),
                                             4, soff, 0, 0, 0);
  }
};


// Bias gradient of the packed QKV projection from the attention backward's per-wave column
// sums: out[seg * H * HD + h * HD + col] = sum over the R rows of head h's partial (seg 0 = q
// with Rq rows, 1 / 2 = k / v with Rk rows).  One 1024-thread block per (seg, head, 16-column
// group): 16 columns x 64 row lanes, then the lanes in a fixed order (deterministic).
template <int HD>
__global__ __launch_bounds__(1024) void attn_bias_grad_k(const float* __restrict__ PQ, const float* __restrict__ PK,
                                                         const float* __restrict__ PV, float* __restrict__ out, int H,
                                                         int Rq, int Rk) {
  constexpr int CG = HD / 16;
  __shared__ float red[64][16];
  const int cgi = blockIdx.x % CG, sh = blockIdx.x / CG, seg = sh / H, h = sh % H;
  const float* P = seg == 0 ? PQ : (seg == 1 ? PK : PV);
  const int R = seg == 0 ? Rq : Rk;
  const int c = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const float* base = P + (long long)h * R * HD + cgi * 16 + c;
  float s = 0.f;
#pragma unroll 8
  for (int r = rl; r < R; r += 64) s += base[(long long)r * HD];
  red[rl][c] = s;
  __syncthreads();
  if (threadIdx.x < 16) {
    float t = 0.f;
    for (int k = 0; k < 64; ++k) t += red[k][threadIdx.x];
    out[(long long)seg * H * HD + (long long)h * HD + cgi * 16 + threadIdx.x] = t;
  }
}


}  // namespace dpfs
