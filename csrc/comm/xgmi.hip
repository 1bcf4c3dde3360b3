// Intra-node tensor-parallel collectives over xGMI peer memory (MI355X, gfx950).
//
// An 8 x MI355X node is a fully connected xGMI mesh: every GPU has one ~153 GB/s link to each of
// its 7 peers.  A ring collective (RCCL's default algorithm for large messages) drives one
// outgoing link per step; the kernels here instead read from all peers at once, so a TP group
// of W ranks keeps all W-1 links busy:
//
//   all-reduce  (two-shot)  copy-in | barrier | rank r sums slice r of every peer's buffer in
//                           fixed rank order (fp32) -> own slice + tmp | barrier | gather the
//                           other W-1 reduced slices from the peers' tmp
//   all-reduce  (one-shot)  copy-in | barrier | every rank reads the WHOLE buffer of every peer
//                           and sums all W in the same fixed rank order (small messages: one
//                           barrier instead of two, (W-1) n bytes read per rank instead of
//                           2 (W-1) n / W; bit-identical to the two-shot result)
//   reduce-scatter          the first two phases of the all-reduce
//   all-gather              copy-in | barrier | read every peer's buffer
//
// Each call runs as ONE kernel on the caller's (side) stream.  Per rank there is one IPC data
// allocation [in | tmp] and one uncached signal allocation; handles are exchanged over the
// c10d store by the Python side (parallel/xgmi.py).  Workgroup b of every rank owns the same
// vector range in every phase, so the barriers are per workgroup: b signals its peers' b and
// waits for their b (no grid-wide barrier, no residency assumption).  Flags are monotonic
// epochs (one per call, identical on every rank because every rank issues the same call
// sequence), compared wrap-safe, never reset.
//
// Memory ordering across GPUs: every byte a peer will read is stored write-through
// (sc0 sc1 buffer stores) and drained (s_waitcnt vmcnt(0)) before a system-scope release and
// the flag store; every remote byte is loaded with sc0 sc1 (system-coherent) buffer loads, so
// neither side depends on L2 state.  Flags are system-scope atomics in uncached memory.
//
// Why the phases are safe without an end barrier: rank r overwrites its `in` region only in
// the copy-in of call k+1, i.e. after its kernel k finished, i.e. after every one of its
// workgroups passed the second barrier of call k, which every peer workgroup signals only after
// its phase-1 reads of `in` completed.  `tmp` is rewritten in phase 1 of call k+1, after the
// start barrier of k+1, which a peer workgroup signals only once that peer's kernel k (and its
// phase-2 reads of tmp) completed (same stream).  The one-shot all-reduce has no second barrier,
// so its input alternates between two regions by the epoch's parity: rank r rewrites region
// (k & 1) only in the copy-in of call k + 2, after passing the start barrier of call k + 1,
// which every peer signals only after its kernel k -- and its reads of r's region -- completed.
//
// Every wait is bounded (s_memrealtime, 100 MHz): on timeout the kernel records an error in a
// host-mapped word and exits, so a broken peer can never hang the GPU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <cstdio>

namespace {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 1024;
constexpr int kThreads = 1024;
constexpr long long kSigBytes = 2LL * kMaxBlocks * kMaxRanks * sizeof(uint32_t);  // [phase][block][src]
constexpr int kAuxSys = 1 | 16;  // sc0 | sc1: system-coherent (write-through stores, L2-bypassing loads)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct Peers {
  char* data[kMaxRanks];     // [in | tmp] of every rank (own included)
  uint32_t* sig[kMaxRanks];  // signal arrays of every rank
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ u32x4 ld_sys(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kAuxSys);
}
__device__ __forceinline__ void st_sys(__amdgpu_buffer_rsrc_t r, unsigned off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kAuxSys);
}

// 16-byte vector <-> fp32 lanes
template <typename T> struct V16;
template <> struct V16<__bf16> {
  static constexpr int N = 8;
  __device__ static void unpack(u32x4 v, float (&f)[8]) {
    bf16x8 b = __builtin_bit_cast(bf16x8, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = (float)b[i];
  }
  __device__ static u32x4 pack(const float (&f)[8]) {
    bf16x8 b;
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = (__bf16)f[i];
    return __builtin_bit_cast(u32x4, b);
  }
};
template <> struct V16<float> {
  static constexpr int N = 4;
  __device__ static void unpack(u32x4 v, float (&f)[4]) {
    f32x4 b = __builtin_bit_cast(f32x4, v);
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = b[i];
  }
  __device__ static u32x4 pack(const float (&f)[4]) {
    f32x4 b;
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = f[i];
    return __builtin_bit_cast(u32x4, b);
  }
};

__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Signal every peer's workgroup `blockIdx.x` (phase p), then wait for all of them.  Lanes
// 0..W-1 of wave 0 each handle one peer.  Returns false on timeout (error recorded).
__device__ __forceinline__ void barrier(const Peers& P, int rank, int W, int phase, uint32_t epoch,
                                        unsigned long long deadline, int* err) {
  drain();           // every wave: its write-through stores have left
  __syncthreads();   // ... for all waves of the workgroup
  const int t = threadIdx.x;
  if (t < W && t != rank) {
    // No L2 write-back is needed (the payload went out write-through and every wave drained
    // it above); the workgroup-scope fences only pin the compiler's ordering.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    uint32_t* f = P.sig[t] + ((size_t)phase * kMaxBlocks + blockIdx.x) * kMaxRanks + rank;
    __hip_atomic_store(f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* mine = P.sig[rank] + ((size_t)phase * kMaxBlocks + blockIdx.x) * kMaxRanks + t;
    while ((int)(__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() > deadline) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    // Remote bytes are read with system-coherent (sc0 sc1) loads, so no cache invalidation is
    // needed here (a system acquire would drop the L2 under the GEMMs running beside us).
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  __syncthreads();
}

// op: 0 all-reduce (x[n] -> out[n], out may alias x), 1 reduce-scatter (x[n] -> out[part]),
//     2 all-gather (x[part] -> out[W*part]).
// n = total elements of the full tensor; part = per-rank slice length (multiple of N).
template <typename T>
__global__ __launch_bounds__(kThreads) void xgmi_coll_k(Peers P, int op, int rank, int W, const T* x, T* out,
                                                       long long n, long long part, long long in_off,
                                                       long long tmp_off, long long cap, uint32_t epoch,
                                                       unsigned long long timeout_ticks, int* err) {
  constexpr int N = V16<T>::N;
  const unsigned long long deadline = __builtin_amdgcn_s_memrealtime() + timeout_ticks;
  const long long nvec = part / N;                       // vectors per slice
  const long long vpb = (nvec + gridDim.x - 1) / gridDim.x;
  const long long v0 = (long long)blockIdx.x * vpb;
  const long long v1 = v0 + vpb < nvec ? v0 + vpb : nvec;
  char* mine = P.data[rank];
  const __amdgpu_buffer_rsrc_t r_in = rsrc(mine + in_off, cap);
  const __amdgpu_buffer_rsrc_t r_tmp = rsrc(mine + tmp_off, cap);
  const u32x4* xv = reinterpret_cast<const u32x4*>(x);
  u32x4* ov = reinterpret_cast<u32x4*>(out);

  // Every loop below issues all of its loads (one per peer) before its first store, so a
  // thread keeps W-1 remote 16-byte reads in flight: with few workgroups (the collective must
  // leave most CUs to the GEMMs running beside it) that is what covers the link latency.
  __amdgpu_buffer_rsrc_t rin[kMaxRanks], rtmp[kMaxRanks];
#pragma unroll
  for (int s = 0; s < kMaxRanks; ++s) {
    rin[s] = rsrc(P.data[s < W ? s : 0] + in_off, cap);
    rtmp[s] = rsrc(P.data[s < W ? s : 0] + tmp_off, cap);
  }

  if (op == 3) {   // one-shot all-reduce: in_off = this call's parity region, whole message
    const long long tv = (n + N - 1) / N;
    const long long bv = (tv + gridDim.x - 1) / gridDim.x;
    const long long w0 = (long long)blockIdx.x * bv, w1 = w0 + bv < tv ? w0 + bv : tv;
    for (long long v = w0 + threadIdx.x; v < w1; v += kThreads) st_sys(r_in, (unsigned)(v * 16), xv[v]);
    barrier(P, rank, W, 0, epoch, deadline, err);
    for (long long v = w0 + threadIdx.x; v < w1; v += kThreads) {
      u32x4 raw[kMaxRanks];
#pragma unroll
      for (int s = 0; s < kMaxRanks; ++s)   // every peer's load before the first add
        if (s < W && s != rank) raw[s] = ld_sys(rin[s], (unsigned)(v * 16));
      const u32x4 self = xv[v];
#pragma unroll
      for (int s = 0; s < kMaxRanks; ++s)
        if (s == rank) raw[s] = self;
      float acc[N], f[N];
      V16<T>::unpack(raw[0], acc);
#pragma unroll
      for (int s = 1; s < kMaxRanks; ++s) {
        if (s < W) {
          V16<T>::unpack(raw[s], f);
#pragma unroll
          for (int i = 0; i < N; ++i) acc[i] += f[i];
        }
      }
      ov[v] = V16<T>::pack(acc);
    }
    return;
  }

  // ---- phase 0: copy-in of what the peers will read.  Staged (op & 8): the producer GEMM
  // wrote x straight into this rank's slot (x == slot base), so nothing is copied; its plain
  // stores may still sit dirty in the XCD L2s, hence a system-scope release (L2 write-back)
  // by one lane of every workgroup before the start barrier (dpfs_xgmi_run launches at least
  // 8 workgroups, which the dispatcher deals one to each XCD).
  const bool staged = (op & 8) != 0;
  op &= 7;
  if (staged) {
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else if (op == 2) {
    for (long long v = v0 + threadIdx.x; v < v1; v += kThreads) st_sys(r_in, (unsigned)(v * 16), xv[v]);
  } else {
    for (long long v = v0 + threadIdx.x; v < v1; v += kThreads) {
      u32x4 c[kMaxRanks];
#pragma unroll
      for (int s = 0; s < kMaxRanks; ++s) {
        const long long e = s * part + v * N;
        if (s < W && s != rank && e < n) c[s] = xv[e / N];
      }
#pragma unroll
      for (int s = 0; s < kMaxRanks; ++s) {
        const long long e = s * part + v * N;
        if (s < W && s != rank && e < n) st_sys(r_in, (unsigned)(e * sizeof(T)), c[s]);
      }
    }
  }
  barrier(P, rank, W, 0, epoch, deadline, err);

  // ---- phase 1
  if (op == 2) {
    for (long long v = v0 + threadIdx.x; v < v1; v += kThreads) {
      u32x4 c[kMaxRanks];
#pragma unroll
      for (int s = 0; s < kMaxRanks; ++s)
        if (s < W) c[s] = (s == rank) ? xv[v] : ld_sys(rin[s], (unsigned)(v * 16));
#pragma unroll
      for (int s = 0; s < kMaxRanks; ++s)
        if (s < W) ov[(s * part) / N + v] = c[s];
    }
  } else {
    const __amdgpu_buffer_rsrc_t* rp = rin;
    const long long base = rank * part;
    for (long long v = v0 + threadIdx.x; v < v1; v += kThreads) {
      const long long e = base + v * N;
      if (e >= n) break;
      u32x4 raw[kMaxRanks];
#pragma unroll
      for (int s = 0; s < kMaxRanks; ++s)   // issue every load before the first add
        if (s < W && s != rank) raw[s] = ld_sys(rp[s], (unsigned)(e * sizeof(T)));
      const u32x4 self = xv[e / N];
#pragma unroll
      for (int s = 0; s < kMaxRanks; ++s)
        if (s == rank) raw[s] = self;
      float acc[N], f[N];
      V16<T>::unpack(raw[0], acc);
#pragma unroll
      for (int s = 1; s < kMaxRanks; ++s) {
        if (s < W) {
          V16<T>::unpack(raw[s], f);
#pragma unroll
          for (int i = 0; i < N; ++i) acc[i] += f[i];
        }
      }
      const u32x4 r = V16<T>::pack(acc);
      if (op == 0) {
        st_sys(r_tmp, (unsigned)(v * 16), r);
        ov[e / N] = r;
      } else {
        ov[v] = r;
      }
    }
  }
  barrier(P, rank, W, 1, epoch, deadline, err);

  // ---- phase 2 (all-reduce): the other ranks' reduced slices
  if (op == 0) {
    for (long long v = v0 + threadIdx.x; v < v1; v += kThreads) {
      u32x4 c[kMaxRanks];
#pragma unroll
      for (int s = 0; s < kMaxRanks; ++s)
        if (s < W && s != rank && s * part + v * N < n) c[s] = ld_sys(rtmp[s], (unsigned)(v * 16));
#pragma unroll
      for (int s = 0; s < kMaxRanks; ++s) {
        const long long e = s * part + v * N;
        if (s < W && s != rank && e < n) ov[e / N] = c[s];
      }
    }
  }
}

struct Comm {
  int rank = 0, world = 1;
  long long cap = 0;          // bytes of each region
  long long os_cap = 0;       // bytes of each of the two one-shot input regions
  int nslots = 0;             // staging slots (producer GEMMs write here: no copy-in)
  char* data = nullptr;       // own [slot 0 .. slot S-1 | stage | tmp], cap bytes each
  uint32_t* sig = nullptr;    // own signals (uncached)
  Peers peers{};
  bool opened[kMaxRanks] = {};
  uint32_t epoch = 0;
  int* err_host = nullptr;
  int* err_dev = nullptr;
  int blocks = 32;
};

thread_local char g_msg[512];

bool ok(hipError_t e, const char* what) {
  if (e == hipSuccess) return true;
  snprintf(g_msg, sizeof(g_msg), "%s: %s", what, hipGetErrorString(e));
  return false;
}

}  // namespace

extern "C" void dpfs_xgmi_destroy(void* h);

extern "C" const char* dpfs_xgmi_last_error() { return g_msg; }

extern "C" long long dpfs_xgmi_handle_bytes() { return 2 * (long long)sizeof(hipIpcMemHandle_t); }

static long long stage_off(const Comm* c) { return (long long)c->nslots * c->cap; }
static long long tmp_off(const Comm* c) { return (long long)(c->nslots + 1) * c->cap; }
static long long os_off(const Comm* c, int parity) { return (long long)(c->nslots + 2) * c->cap + parity * c->os_cap; }
static const long long kOneShotCap = 16LL << 20;   // one-shot all-reduce: messages up to 16 MiB

// Allocate this rank's buffers; writes [data handle | signal handle] to handles_out.
extern "C" void* dpfs_xgmi_create(int rank, int world, long long cap_bytes, int nslots, void* handles_out) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world) {
    snprintf(g_msg, sizeof(g_msg), "xgmi: world %d / rank %d out of range (max %d ranks)", world, rank, kMaxRanks);
    return nullptr;
  }
  if (cap_bytes <= 0 || cap_bytes >= (1LL << 31) || cap_bytes % 4096) {
    snprintf(g_msg, sizeof(g_msg), "xgmi: capacity %lld must be a positive multiple of 4096 below 2 GiB", cap_bytes);
    return nullptr;
  }
  if (nslots < 0 || nslots > 16) {
    snprintf(g_msg, sizeof(g_msg), "xgmi: %d staging slots (0..16)", nslots);
    return nullptr;
  }
  Comm* c = new Comm();
  c->rank = rank;
  c->world = world;
  c->cap = cap_bytes;
  c->nslots = nslots;
  c->os_cap = cap_bytes < kOneShotCap ? cap_bytes : kOneShotCap;
  if (!ok(hipMalloc((void**)&c->data, (nslots + 2) * cap_bytes + 2 * c->os_cap), "hipMalloc(data)")) {
    delete c;
    return nullptr;
  }
  // Signals: uncached device memory when it can be IPC-exported, plain device memory otherwise
  // (every signal access is a system-scope atomic either way).
  hipIpcMemHandle_t hs;
  if (hipExtMallocWithFlags((void**)&c->sig, kSigBytes, hipDeviceMallocUncached) != hipSuccess ||
      hipIpcGetMemHandle(&hs, c->sig) != hipSuccess) {
    (void)hipGetLastError();
    if (c->sig) (void)hipFree(c->sig);
    c->sig = nullptr;
    if (!ok(hipMalloc((void**)&c->sig, kSigBytes), "hipMalloc(sig)") ||
        !ok(hipIpcGetMemHandle(&hs, c->sig), "hipIpcGetMemHandle(sig)")) {
      dpfs_xgmi_destroy(c);
      return nullptr;
    }
  }
  if (!ok(hipMemset(c->sig, 0, kSigBytes), "hipMemset(sig)") ||
      !ok(hipHostMalloc((void**)&c->err_host, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent),
          "hipHostMalloc(err)") ||
      !ok(hipHostGetDevicePointer((void**)&c->err_dev, c->err_host, 0), "hipHostGetDevicePointer(err)")) {
    dpfs_xgmi_destroy(c);
    return nullptr;
  }
  *c->err_host = 0;
  hipIpcMemHandle_t hd;
  if (!ok(hipIpcGetMemHandle(&hd, c->data), "hipIpcGetMemHandle(data)")) {
    dpfs_xgmi_destroy(c);
    return nullptr;
  }
  memcpy(handles_out, &hd, sizeof(hd));
  memcpy((char*)handles_out + sizeof(hd), &hs, sizeof(hs));
  c->peers.data[rank] = c->data;
  c->peers.sig[rank] = c->sig;
  if (!ok(hipDeviceSynchronize(), "hipDeviceSynchronize")) {
    dpfs_xgmi_destroy(c);
    return nullptr;
  }
  return c;
}

// handles: world x [data handle | signal handle], in rank order.
extern "C" int dpfs_xgmi_open(void* h, const void* handles) {
  Comm* c = (Comm*)h;
  const long long hb = dpfs_xgmi_handle_bytes();
  for (int r = 0; r < c->world; ++r) {
    if (r == c->rank) continue;
    hipIpcMemHandle_t hd, hs;
    memcpy(&hd, (const char*)handles + r * hb, sizeof(hd));
    memcpy(&hs, (const char*)handles + r * hb + sizeof(hd), sizeof(hs));
    void *pd = nullptr, *ps = nullptr;
    if (!ok(hipIpcOpenMemHandle(&pd, hd, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(data)")) return -1;
    if (!ok(hipIpcOpenMemHandle(&ps, hs, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(sig)")) return -1;
    c->peers.data[r] = (char*)pd;
    c->peers.sig[r] = (uint32_t*)ps;
    c->opened[r] = true;
  }
  return 0;
}

extern "C" void dpfs_xgmi_set_blocks(void* h, int blocks) {
  Comm* c = (Comm*)h;
  c->blocks = blocks < 1 ? 1 : (blocks > kMaxBlocks ? kMaxBlocks : blocks);
}

extern "C" long long dpfs_xgmi_capacity(void* h) { return ((Comm*)h)->cap; }
extern "C" long long dpfs_xgmi_one_shot_capacity(void* h) { return ((Comm*)h)->os_cap; }

// Device address of staging slot `slot` (cap bytes), or null.
extern "C" void* dpfs_xgmi_slot(void* h, int slot) {
  Comm* c = (Comm*)h;
  return (slot >= 0 && slot < c->nslots) ? c->data + (long long)slot * c->cap : nullptr;
}

// Host-visible error word (1 = a barrier timed out).  Reading it does not synchronise.
extern "C" int dpfs_xgmi_error(void* h) { return __atomic_load_n(((Comm*)h)->err_host, __ATOMIC_RELAXED); }

extern "C" void dpfs_xgmi_clear_error(void* h) { __atomic_store_n(((Comm*)h)->err_host, 0, __ATOMIC_RELAXED); }

// One collective on `stream`.  dtype 1 = bf16, 0 = fp32.  Element counts as in xgmi_coll_k;
// the caller guarantees n*elt <= cap (op 0/1) / W*part*elt <= ... (op 2: part*elt <= cap) and
// 16-byte alignment of x and out.  op 3 = one-shot all-reduce (n*elt <= the one-shot capacity,
// never staged: peers read the input after this rank's kernel may have finished).
extern "C" int dpfs_xgmi_run(void* h, int op, int dtype, const void* x, void* out, long long n, long long part,
                             double timeout_s, int slot, hipStream_t stream) {
  Comm* c = (Comm*)h;
  if (op == 3) {
    const int elt1 = dtype == 1 ? 2 : 4;
    const long long nb = ((n * elt1 + 15) / 16) * 16;
    if (slot >= 0 || n <= 0 || nb > c->os_cap || (n * elt1) % 16) {
      snprintf(g_msg, sizeof(g_msg), "xgmi_run: one-shot all-reduce of %lld B (one-shot capacity %lld B, unstaged, "
               "16-byte multiple)", n * elt1, c->os_cap);
      return -1;
    }
    const long long tv = nb / 16;
    int grid = (int)((tv + kThreads - 1) / kThreads);
    if (grid > c->blocks) grid = c->blocks;
    if (grid < 1) grid = 1;
    c->epoch += 1;
    if (c->epoch == 0) c->epoch = 1;
    const unsigned long long ticks = (unsigned long long)(timeout_s * 1e8);
    const long long io = os_off(c, (int)(c->epoch & 1));
    if (dtype == 1)
      hipLaunchKernelGGL(xgmi_coll_k<__bf16>, dim3(grid), dim3(kThreads), 0, stream, c->peers, 3, c->rank, c->world,
                         (const __bf16*)x, (__bf16*)out, n, n, io, tmp_off(c), c->os_cap, c->epoch, ticks, c->err_dev);
    else
      hipLaunchKernelGGL(xgmi_coll_k<float>, dim3(grid), dim3(kThreads), 0, stream, c->peers, 3, c->rank, c->world,
                         (const float*)x, (float*)out, n, n, io, tmp_off(c), c->os_cap, c->epoch, ticks, c->err_dev);
    return ok(hipGetLastError(), "xgmi_coll_k launch") ? 0 : -1;
  }
  long long in_off = stage_off(c);
  if (slot >= 0) {   // staged input: x must be the slot itself (reduce-scatter / all-reduce)
    if (slot >= c->nslots || x != c->data + (long long)slot * c->cap || op == 2) {
      snprintf(g_msg, sizeof(g_msg), "xgmi_run: staged input must start at slot %d (all-reduce / reduce-scatter)",
               slot);
      return -1;
    }
    in_off = (long long)slot * c->cap;
  }
  const int elt = dtype == 1 ? 2 : 4;
  const int N = 16 / elt;
  if (part % N || (op == 2 ? part * elt > c->cap : ((n + N - 1) / N) * N * elt > c->cap) || n <= 0) {
    snprintf(g_msg, sizeof(g_msg), "xgmi_run: bad sizes n=%lld part=%lld (cap %lld B)", n, part, c->cap);
    return -1;
  }
  const long long nvec = part / N;
  int grid = (int)((nvec + kThreads - 1) / kThreads);
  if (grid > c->blocks) grid = c->blocks;
  // At least one workgroup per XCD (workgroups are dealt round-robin over the 8 XCDs): the
  // staged path's system-scope release writes back the L2 of the XCD it runs on only, and the
  // producer GEMM's dirty lines may sit in any XCD's L2.  Applied to every call (not only the
  // staged ones) so the grid is a function of the size alone, identical on every rank.
  const int min_grid = c->blocks < 8 ? c->blocks : 8;
  if (grid < min_grid) grid = min_grid;
  if (grid < 1) grid = 1;
  c->epoch += 1;
  if (c->epoch == 0) c->epoch = 1;
  const unsigned long long ticks = (unsigned long long)(timeout_s * 1e8);  // s_memrealtime: 100 MHz
  const int kop = op | (slot >= 0 ? 8 : 0);
  if (dtype == 1)
    hipLaunchKernelGGL(xgmi_coll_k<__bf16>, dim3(grid), dim3(kThreads), 0, stream, c->peers, kop, c->rank, c->world,
                       (const __bf16*)x, (__bf16*)out, n, part, in_off, tmp_off(c), c->cap, c->epoch, ticks,
                       c->err_dev);
  else
    hipLaunchKernelGGL(xgmi_coll_k<float>, dim3(grid), dim3(kThreads), 0, stream, c->peers, kop, c->rank, c->world,
                       (const float*)x, (float*)out, n, part, in_off, tmp_off(c), c->cap, c->epoch, ticks,
                       c->err_dev);
  return ok(hipGetLastError(), "xgmi_coll_k launch") ? 0 : -1;
}

extern "C" void dpfs_xgmi_destroy(void* h) {
  Comm* c = (Comm*)h;
  if (!c) return;
  (void)hipDeviceSynchronize();
  for (int r = 0; r < c->world; ++r) {
    if (!c->opened[r]) continue;
    (void)hipIpcCloseMemHandle(c->peers.data[r]);
    (void)hipIpcCloseMemHandle(c->peers.sig[r]);
  }
  if (c->data) (void)hipFree(c->data);
  if (c->sig) (void)hipFree(c->sig);
  if (c->err_host) (void)hipHostFree(c->err_host);
  delete c;
}
