// Python bindings of the gfx950 kernels: torch tensors in, kernels launched on the current
// HIP stream (so they interleave correctly with RCCL collectives issued by
// torch.distributed on its own streams and with hipGraph capture).
//
// Every function validates device/dtype/shape/stride assumptions of its kernel on the host
// BEFORE launching (an out-of-bounds wave can reset the whole node), allocates outputs from
// the PyTorch caching allocator, and mirrors the signature of the pure-PyTorch oracle of
// the same name in distributed_pytorch_from_scratch_amd/ops/reference.py.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <ATen/DeviceGuard.h>
#include <hip/hip_runtime.h>

#include <vector>

extern "C" {
void dpfs_gemm_nt(const void*, const void*, void*, const float*, int, int, int, int, int, int, int, hipStream_t);
void dpfs_gemm_nn(const void*, const void*, void*, int, int, int, int, int, int, int, hipStream_t);
int dpfs_gemm_tn_splits(int, int, int);
long long dpfs_gemm_tn_group_ws(int, const int*, const int*, const int*, const int*, int, const int*, const int*,
                                 const int*, int);
int dpfs_gemm_tn_group(int, const void* const*, const void* const*, float* const*, const int*, const int*, const int*,
                       const int*, const int*, int, float*, long long, const void* const*, const void* const*,
                       const int*, const int*, int, hipStream_t);
long long dpfs_gemm_tn_ws(int, int, int, int);
void dpfs_gemm_set_impl(int);
int dpfs_gemm_rope_fusable(int, int, int, int, int);
void dpfs_gemm_nt_rope(const void*, const void*, void*, const float*, int, int, int, int, int, int, const int64_t*,
                       const float*, int, int, int, hipStream_t);
void dpfs_gemm4_sched(int);
void dpfs_gemm4_br(int);
void dpfs_gemm4_br_tn(int);
void dpfs_gemm4_m32(int);
void dpfs_attn_prefetch(int);
void dpfs_gemm4_swb_depth(int);
void dpfs_gemm4_m32k(int);
void dpfs_gemm4_group_m(int);
void dpfs_gemm4_ablate(int);
void dpfs_gemm4_diag(void*);
void dpfs_attn_diag(void*);
void dpfs_gemm_force(int, int);
void dpfs_gemm_v2_sched(int);
void dpfs_gemm_set_workspace(float*, long long);
long long dpfs_gemm_bf16_ws(int, int, int);
long long dpfs_gemm4_sk_ws(int, int, int);
int dpfs_gemm4_sk_error(int);
void dpfs_gemm4_sk_starve(int);
void dpfs_gemm_tn(const void*, const void*, float*, float*, int, int, int, int, int, int, int, hipStream_t);
int dpfs_gemm_tn2(const void*, const void*, const void*, const void*, float*, float*, int, int, int, int, int, int, int,
                  int, int, int, hipStream_t);
long long dpfs_gemm_tn2_ws(int, int, int, int);
void dpfs_rmsnorm_fwd(int, const void*, const float*, void*, float*, int, int, float, hipStream_t);
void dpfs_layernorm_fwd(int, const void*, const float*, const float*, void*, float*, float*, int, int, float,
                        hipStream_t);
int dpfs_norm_bwd_grid(int);
void dpfs_norm_bwd(int, int, const void*, const void*, const float*, const float*, const float*, const void*, void*,
                   float*, float*, float*, float*, int, int, hipStream_t);
void dpfs_swiglu_fwd(int, const void*, void*, int, int, int, hipStream_t);
void dpfs_swiglu_bwd(int, const void*, const void*, void*, int, int, int, hipStream_t);
long long dpfs_swiglu_bwd_dbias_ws(int, int);
void dpfs_swiglu_bwd_dbias(int, const void*, const void*, void*, float*, float*, int, int, int, hipStream_t);
void dpfs_colsum_rows_small(const float*, float*, int, int, hipStream_t);
bool dpfs_gemm4_nn_swiglu_bwd(const void*, const void*, const void*, void*, float*, int, int, int, int, int, int, int,
                              int, unsigned, unsigned, hipStream_t);
bool dpfs_gemm4_nt_swiglu(const void*, const void*, void*, const float*, void*, int, int, int, int, int, int, int,
                          unsigned, unsigned, hipStream_t);
long long dpfs_ce_bwd_dbias_ws(int, int, int);
void dpfs_ce_bwd_dbias(int, const void*, const int64_t*, const float*, const float*, void*, float*, float*, int, int,
                       long long, int, hipStream_t);
void dpfs_rope(int, void*, const int64_t*, const float*, int, int, int, int, int, hipStream_t);
void dpfs_bias_residual(int, const void*, const float*, const void*, void*, int, int, hipStream_t);
long long dpfs_colsum_ws(int, int);
long long dpfs_norm_bwd_ws(int, int, int);
void dpfs_add_rmsnorm_fwd(int, const void*, const float*, const void*, const float*, void*, void*, float*, int, int,
                          float, hipStream_t);
int dpfs_norm_bwd_grid(int);
void dpfs_bias_grad(int, const void*, float*, float*, int, int, hipStream_t);
void dpfs_embedding_fwd(int, const int64_t*, const float*, void*, int, int, long long, int, hipStream_t);
void dpfs_embedding_bwd(int, const void*, const int64_t*, float*, int, int, long long, int, hipStream_t);
void dpfs_embedding_bwd_seg(int, const void*, const int64_t*, const int64_t*, float*, int, int, int, hipStream_t);
void dpfs_ce_stats(int, const void*, const int64_t*, float*, int, int, long long, int, hipStream_t);
long long dpfs_ce_fused_ws(int, int);
int dpfs_ce_fused(int, void*, const int64_t*, const float*, float*, float*, float*, int, int, long long, int,
                  hipStream_t);
void dpfs_ce_bwd(int, const void*, const int64_t*, const float*, const float*, void*, int, int, long long, int,
                 hipStream_t);
int dpfs_adam_chunk();
int dpfs_adam_desc_bytes();
void dpfs_adam_step(const void*, const int*, int, float, float, float, float, float, float, float, float, const float*,
                    hipStream_t);
void dpfs_grad_sumsq(const void*, const int*, int, float*, hipStream_t);
int dpfs_attn_supported_hd(int);
void dpfs_attn_fwd(const void*, const void*, const void*, void*, float*, int, int, int, int, long long, long long,
                   long long, long long, float, int, int, hipStream_t);
int dpfs_attn_bwd(const void*, const void*, const void*, const void*, const void*, const float*, float*, void*, void*,
                   void*, int, int, int, int, long long, long long, long long, long long, long long, long long,
                   long long, long long, float, int, const int64_t*, const float*, hipStream_t, float*, float*, int);
long long dpfs_attn_bias_ws(int, int, int, int);
int dpfs_ce_part_floats();
void dpfs_ce_finalize(const float*, const int64_t*, long long, float*, float*, float*, float*, float*, int, int, int,
                      int, hipStream_t);
void dpfs_ce_valid_scale(const int64_t*, long long, float*, float*, float*, int, hipStream_t);
void dpfs_ce_grad_scale(const float*, const void*, int, const float*, float*, int, hipStream_t);
long long dpfs_emb_sort_ws(int);
void dpfs_occupy(int, double, hipStream_t);
void dpfs_attn_stagger(int);
void dpfs_gemm_f32(int, const void*, const void*, void*, const float*, int, int, int, long long, long long,
                   long long, int, float*, int, int, hipStream_t);
int dpfs_gemm_f32_splits(int, int, int);
int dpfs_attn_f32_supported_hd(int);
void dpfs_attn_fwd_f32(const float*, const float*, const float*, float*, float*, int, int, int, int, long long,
                       long long, long long, long long, float, int, hipStream_t);
long long dpfs_attn_bwd_f32_ws(int, int, int, int, int);
int dpfs_attn_bwd_f32(const float*, const float*, const float*, const float*, const float*, const float*, float*,
                      float*, float*, float*, int, int, int, int, long long, long long, long long, long long, long long,
                      long long, long long, long long, float, int, const int64_t*, const float*, float*, hipStream_t);
void dpfs_emb_sort(const int64_t*, int, long long, int, int*, int64_t*, int64_t*, hipStream_t);
long long dpfs_attn_fused_ws(int, int, int, int);
long long dpfs_attn_fused_bias_ws(int, int, int, int);
int dpfs_attn_bwd_fused(const void*, const void*, const void*, const void*, const void*, const float*, float*, float*,
                        void*, void*, void*, int, int, int, int, long long, long long, long long, long long, long long,
                        long long, long long, long long, float, int, const int64_t*, const float*, hipStream_t, float*,
                        float*);
// kernels/decode.hip
int dpfs_decode_nsplit(int);
void dpfs_attn_decode(const void*, long long, const void*, const void*, const int*, void*, long long, float*, int, int,
                      int, int, float, hipStream_t);
void dpfs_kv_append(const void*, const void*, long long, void*, void*, const int*, int, int, int, int, hipStream_t);
void dpfs_step_advance(int*, int64_t*, int, hipStream_t);
void dpfs_fp8_quant(const void*, long long, int, void*, float*, float*, hipStream_t);
int dpfs_fp8_work_floats();
int dpfs_gemv16_ok(int, int, int, long long, long long);
void dpfs_gemv16(const void*, long long, const void*, long long, const float*, void*, long long, int, int, int, int,
                 hipStream_t);
void dpfs_rope_append(void*, long long, const int64_t*, const float*, void*, void*, const int*, int, int, int, int,
                      hipStream_t);
// comm/xgmi.hip
const char* dpfs_xgmi_last_error();
long long dpfs_xgmi_handle_bytes();
void* dpfs_xgmi_create(int, int, long long, int, void*);
void* dpfs_xgmi_slot(void*, int);
int dpfs_xgmi_open(void*, const void*);
void dpfs_xgmi_set_blocks(void*, int);
long long dpfs_xgmi_capacity(void*);
long long dpfs_xgmi_one_shot_capacity(void*);
int dpfs_xgmi_error(void*);
void dpfs_xgmi_clear_error(void*);
int dpfs_xgmi_run(void*, int, int, const void*, void*, long long, long long, double, int, hipStream_t);
void dpfs_xgmi_destroy(void*);
void dpfs_adam_patch_grads(void*, const long long*, int, hipStream_t);
// blas/blaslt.hip
const char* dpfs_lt_last_error();
int dpfs_lt_algos(int, long long, long long, long long, int);
long long dpfs_lt_workspace(int, long long, long long, long long, int, int);
int dpfs_lt_run(int, long long, long long, long long, const float*, int, const void*, const void*, void*, float, void*,
                long long, hipStream_t);
// comm/rccl_comm.hip
const char* dpfs_rccl_last_error();
int dpfs_rccl_id_bytes();
int dpfs_rccl_unique_id(void*);
int dpfs_rccl_init(const void*, int, int, void**);
int dpfs_rccl_destroy(void*);
int dpfs_rccl_async_error(void*);
int dpfs_rccl_all_reduce(void*, const void*, void*, size_t, int, int, hipStream_t);
int dpfs_rccl_reduce_scatter(void*, const void*, void*, size_t, int, int, hipStream_t);
int dpfs_rccl_all_gather(void*, const void*, void*, size_t, int, hipStream_t);
int dpfs_rccl_broadcast(void*, const void*, void*, size_t, int, int, hipStream_t);
int dpfs_rccl_group_start();
int dpfs_rccl_group_end();
}

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

int dcode(const torch::Tensor& t) {
  if (t.scalar_type() == torch::kBFloat16) return 1;
  if (t.scalar_type() == torch::kFloat32) return 0;
  TORCH_CHECK(false, "unsupported dtype ", t.scalar_type(), " (bf16 / fp32 only)");
  return -1;
}

void check_cuda(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a HIP (cuda) tensor");
}

void check_rowmajor(const torch::Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.dim() == 2, name, " must be 2-D, got ", t.dim(), "-D");
  TORCH_CHECK(t.stride(1) == 1, name, " must have unit inner stride");
}

const float* opt_f32(const c10::optional<torch::Tensor>& t, int64_t n, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_cuda(*t, name);
  TORCH_CHECK(t->scalar_type() == torch::kFloat32 && t->is_contiguous() && t->numel() == n, name,
              " must be a contiguous fp32 vector of length ", n);
  return t->data_ptr<float>();
}

// -------------------------------------------------------------------------------- GEMM --
torch::Tensor rope_(torch::Tensor qkv, torch::Tensor positions, torch::Tensor table, int64_t n_rot_heads,
                    int64_t head_dim, bool inverse);

// Output buffer: `out` when given (contiguous [M, N] of a's dtype, e.g. a staging slot of the
// xGMI collectives), else a fresh tensor.
torch::Tensor gemm_out(const c10::optional<torch::Tensor>& out, const torch::Tensor& a, int64_t M, int64_t N) {
  if (!out.has_value() || !out->defined()) return torch::empty({M, N}, a.options());
  check_cuda(*out, "out");
  TORCH_CHECK(out->is_contiguous() && out->dim() == 2 && out->size(0) == M && out->size(1) == N &&
                  out->scalar_type() == a.scalar_type(),
              "gemm: out must be a contiguous [M, N] tensor of the operand dtype");
  return *out;
}

// NT output: `out` may also be a row-major column slice of a wider buffer (unit column stride,
// row stride >= N and a multiple of 8), e.g. the V columns of the packed QKV output.
torch::Tensor gemm_out_rows(const c10::optional<torch::Tensor>& out, const torch::Tensor& a, int64_t M, int64_t N) {
  if (!out.has_value() || !out->defined()) return torch::empty({M, N}, a.options());
  check_cuda(*out, "out");
  TORCH_CHECK(out->dim() == 2 && out->size(0) == M && out->size(1) == N && out->scalar_type() == a.scalar_type() &&
                  (N <= 1 || out->stride(1) == 1) && out->stride(0) >= N && out->stride(0) % 8 == 0,
              "gemm_nt: out must be a row-major [M, N] tensor (or column slice) of the operand dtype");
  return *out;
}

torch::Tensor gemm_nt(torch::Tensor a, torch::Tensor b, c10::optional<torch::Tensor> bias,
                      c10::optional<torch::Tensor> rope_pos, c10::optional<torch::Tensor> rope_tab,
                      int64_t rope_heads, int64_t rope_hd, c10::optional<torch::Tensor> out, int64_t variant) {
  check_rowmajor(a, "a");
  TORCH_CHECK((variant >= 0 && variant <= 6) || variant == 8 || variant == 12,
              "gemm: variant 0 (v4), 1 (v4 256-wide), 2 (v4 192-wide), 3 (v3), 8 (v4 stream-K 256-wide); "
              "+4: v4 with non-temporal output stores");
  check_rowmajor(b, "b");
  TORCH_CHECK(a.scalar_type() == torch::kBFloat16 && b.scalar_type() == torch::kBFloat16, "gemm_nt: bf16 operands");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K, "gemm_nt: K mismatch ", K, " vs ", b.size(1));
  TORCH_CHECK(K % 8 == 0, "gemm_nt: K must be a multiple of 8, got ", K);
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0, "gemm_nt: row strides must be multiples of 8");
  const at::DeviceGuard g(a.device());
  auto c = gemm_out_rows(out, a, M, N);
  if (M == 0 || N == 0) return c;
  if (K == 0) return c.zero_();
  TORCH_CHECK(N % 4 == 0, "gemm_nt: N must be a multiple of 4, got ", N);
  const int ldc = (int)(M > 1 ? c.stride(0) : N);
  long long wsn = dpfs_gemm_bf16_ws((int)M, (int)N, (int)K);
  if (variant & 8) {   // stream-K (where it applies: it replaces the split-K slabs) -- its partials / flags
    const long long skn = dpfs_gemm4_sk_ws((int)M, (int)N, (int)K);
    if (skn > 0) wsn = skn;
  }
  torch::Tensor ws;
  if (wsn > 0) ws = torch::empty({wsn}, a.options().dtype(torch::kFloat32));
  dpfs_gemm_set_workspace(wsn > 0 ? ws.data_ptr<float>() : nullptr, wsn);
  const bool want_rope = rope_pos.has_value() && rope_pos->defined() && rope_heads > 0;
  if (want_rope && dpfs_gemm_rope_fusable((int)M, (int)N, (int)K, (int)rope_hd, (int)variant)) {
    TORCH_CHECK(rope_pos->scalar_type() == torch::kInt64 && rope_pos->is_contiguous() && rope_pos->numel() == M,
                "gemm_nt: rope_pos must be contiguous int64 [M]");
    TORCH_CHECK(rope_tab.has_value() && rope_tab->scalar_type() == torch::kFloat32 && rope_tab->is_contiguous() &&
                    rope_tab->size(1) == rope_hd,
                "gemm_nt: rope_tab must be fp32 [maxlen, hd]");
    dpfs_gemm_nt_rope(a.data_ptr(), b.data_ptr(), c.data_ptr(), opt_f32(bias, N, "bias"), (int)M, (int)N, (int)K,
                      (int)a.stride(0), (int)b.stride(0), ldc, rope_pos->data_ptr<int64_t>(),
                      rope_tab->data_ptr<float>(), (int)(rope_heads * rope_hd), (int)rope_hd, (int)variant, stream());
  } else {
    TORCH_CHECK(!want_rope || ldc == N, "gemm_nt: the separate RoPE pass needs a contiguous output");
    dpfs_gemm_nt(a.data_ptr(), b.data_ptr(), c.data_ptr(), opt_f32(bias, N, "bias"), (int)M, (int)N, (int)K,
                 (int)a.stride(0), (int)b.stride(0), ldc, (int)variant, stream());
    if (want_rope) rope_(c, *rope_pos, *rope_tab, rope_heads, rope_hd, false);
  }
  dpfs_gemm_set_workspace(nullptr, 0);
  return c;
}

torch::Tensor gemm_nn(torch::Tensor a, torch::Tensor b, c10::optional<torch::Tensor> out, int64_t variant) {
  check_rowmajor(a, "a");
  TORCH_CHECK((variant >= 0 && variant <= 6) || variant == 8 || variant == 12,
              "gemm: variant 0 (v4), 1 (v4 256-wide), 2 (v4 192-wide), 3 (v3), 8 (v4 stream-K 256-wide); "
              "+4: v4 with non-temporal output stores");
  check_rowmajor(b, "b");
  TORCH_CHECK(a.scalar_type() == torch::kBFloat16 && b.scalar_type() == torch::kBFloat16, "gemm_nn: bf16 operands");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(1);
  TORCH_CHECK(b.size(0) == K, "gemm_nn: K mismatch");
  TORCH_CHECK(K % 8 == 0 && N % 8 == 0, "gemm_nn: K and N must be multiples of 8, got ", K, " ", N);
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0, "gemm_nn: row strides must be multiples of 8");
  const at::DeviceGuard g(a.device());
  auto c = gemm_out(out, a, M, N);
  if (M == 0 || N == 0) return c;
  if (K == 0) return c.zero_();
  long long wsn = dpfs_gemm_bf16_ws((int)M, (int)N, (int)K);
  if (variant & 8) {   // stream-K (where it applies: it replaces the split-K slabs) -- its partials / flags
    const long long skn = dpfs_gemm4_sk_ws((int)M, (int)N, (int)K);
    if (skn > 0) wsn = skn;
  }
  torch::Tensor ws;
  if (wsn > 0) ws = torch::empty({wsn}, a.options().dtype(torch::kFloat32));
  dpfs_gemm_set_workspace(wsn > 0 ? ws.data_ptr<float>() : nullptr, wsn);
  dpfs_gemm_nn(a.data_ptr(), b.data_ptr(), c.data_ptr(), (int)M, (int)N, (int)K, (int)a.stride(0), (int)b.stride(0),
               (int)N, (int)variant, stream());
  dpfs_gemm_set_workspace(nullptr, 0);
  return c;
}

// c[M,N] fp32 = a[K,M]^T b[K,N]
torch::Tensor gemm_tn(torch::Tensor a, torch::Tensor b, c10::optional<torch::Tensor> out, bool accumulate,
                      int64_t variant) {
  check_rowmajor(a, "a");
  TORCH_CHECK(variant == 0 || variant == 3, "gemm_tn: variant 0 (v4) or 3 (v3)");
  check_rowmajor(b, "b");
  TORCH_CHECK(a.scalar_type() == torch::kBFloat16 && b.scalar_type() == torch::kBFloat16, "gemm_tn: bf16 operands");
  const int64_t K = a.size(0), M = a.size(1), N = b.size(1);
  TORCH_CHECK(b.size(0) == K, "gemm_tn: K mismatch");
  TORCH_CHECK(M % 8 == 0 && N % 8 == 0, "gemm_tn: M and N must be multiples of 8, got ", M, " ", N);
  TORCH_CHECK(a.stride(0) % 8 == 0 && b.stride(0) % 8 == 0, "gemm_tn: row strides must be multiples of 8");
  const at::DeviceGuard g(a.device());
  torch::Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    TORCH_CHECK(c.scalar_type() == torch::kFloat32 && c.is_contiguous() && c.size(0) == M && c.size(1) == N,
                "gemm_tn: out must be contiguous fp32 [M,N]");
  } else {
    c = torch::empty({M, N}, a.options().dtype(torch::kFloat32));
    accumulate = false;
  }
  if (M == 0 || N == 0) return c;
  if (K == 0) {
    if (!accumulate) c.zero_();
    return c;
  }
  const long long wsn = dpfs_gemm_tn_ws((int)M, (int)N, (int)K, accumulate ? 1 : 0);
  torch::Tensor ws;
  if (wsn > 0) ws = torch::empty({(int64_t)wsn}, c.options());
  dpfs_gemm_tn(a.data_ptr(), b.data_ptr(), c.data_ptr<float>(), ws.defined() ? ws.data_ptr<float>() : nullptr, (int)M,
               (int)N, (int)K, (int)a.stride(0), (int)b.stride(0), accumulate ? 1 : 0, (int)variant, stream());
  return c;
}

// outs[g] fp32 (+= when acc[g]) a[g][K, M_g]^T b[g][K, N_g] for up to 4 GEMMs over one K as
// one grouped launch (+ one reduction); with a2 / b2 the rows continue in second buffers
// (a chunked step's other ping-pong chunk, K1 rows each).  False (nothing written) where the
// group does not apply.
bool gemm_tn_group(std::vector<torch::Tensor> a, std::vector<torch::Tensor> b, std::vector<torch::Tensor> outs,
                   std::vector<int64_t> acc, c10::optional<std::vector<torch::Tensor>> a2,
                   c10::optional<std::vector<torch::Tensor>> b2) {
  const size_t n = a.size();
  TORCH_CHECK(n >= 1 && n <= 4 && b.size() == n && outs.size() == n && acc.size() == n, "gemm_tn_group: 1..4 GEMMs");
  const bool two = a2.has_value() && b2.has_value();
  TORCH_CHECK(!two || (a2->size() == n && b2->size() == n), "gemm_tn_group: a2 / b2 per GEMM");
  const int64_t K = a[0].size(0);
  const int64_t K1 = two ? (*a2)[0].size(0) : 0;
  const void* pa[4];
  const void* pb[4];
  const void* pa2[4] = {nullptr, nullptr, nullptr, nullptr};
  const void* pb2[4] = {nullptr, nullptr, nullptr, nullptr};
  float* pc[4];
  int M[4], N[4], lda[4], ldb[4], ac[4], lda2[4] = {0, 0, 0, 0}, ldb2[4] = {0, 0, 0, 0};
  for (size_t g = 0; g < n; ++g) {
    check_rowmajor(a[g], "gemm_tn_group a");
    check_rowmajor(b[g], "gemm_tn_group b");
    TORCH_CHECK(a[g].scalar_type() == torch::kBFloat16 && b[g].scalar_type() == torch::kBFloat16,
                "gemm_tn_group: bf16 operands");
    TORCH_CHECK(a[g].size(0) == K && b[g].size(0) == K, "gemm_tn_group: one K for the group");
    TORCH_CHECK(a[g].device() == a[0].device() && b[g].device() == a[0].device() && outs[g].device() == a[0].device(),
                "gemm_tn_group: one device");
    M[g] = (int)a[g].size(1);
    N[g] = (int)b[g].size(1);
    TORCH_CHECK(outs[g].scalar_type() == torch::kFloat32 && outs[g].is_contiguous() && outs[g].dim() == 2 &&
                    outs[g].size(0) == M[g] && outs[g].size(1) == N[g],
                "gemm_tn_group: out must be contiguous fp32 [M,N]");
    lda[g] = (int)a[g].stride(0);
    ldb[g] = (int)b[g].stride(0);
    ac[g] = acc[g] ? 1 : 0;
    pa[g] = a[g].data_ptr();
    pb[g] = b[g].data_ptr();
    pc[g] = outs[g].data_ptr<float>();
    if (two) {
      const torch::Tensor& x = (*a2)[g];
      const torch::Tensor& y = (*b2)[g];
      check_rowmajor(x, "gemm_tn_group a2");
      check_rowmajor(y, "gemm_tn_group b2");
      TORCH_CHECK(x.scalar_type() == torch::kBFloat16 && y.scalar_type() == torch::kBFloat16 && x.size(0) == K1 &&
                      y.size(0) == K1 && x.size(1) == M[g] && y.size(1) == N[g] && x.device() == a[0].device() &&
                      y.device() == a[0].device(),
                  "gemm_tn_group: a2 [K1, M] / b2 [K1, N] bf16 on the group's device");
      lda2[g] = (int)x.stride(0);
      ldb2[g] = (int)y.stride(0);
      pa2[g] = x.data_ptr();
      pb2[g] = y.data_ptr();
    }
  }
  if (K <= 0 || K + K1 >= (1ll << 31) || (two && K1 <= 0)) return false;
  const long long wsn = dpfs_gemm_tn_group_ws((int)n, M, N, lda, ldb, (int)K, ac, two ? lda2 : nullptr,
                                              two ? ldb2 : nullptr, (int)K1);
  if (wsn < 0) return false;
  const at::DeviceGuard dg(a[0].device());
  torch::Tensor ws;
  if (wsn > 0) ws = torch::empty({(int64_t)wsn}, outs[0].options());
  return dpfs_gemm_tn_group((int)n, pa, pb, pc, M, N, lda, ldb, ac, (int)K, ws.defined() ? ws.data_ptr<float>() : nullptr,
                            wsn, pa2, pb2, lda2, ldb2, (int)K1, stream()) != 0;
}

// c[M,N] fp32 (+)= a0[K0,M]^T b0[K0,N] + a1[K1,M]^T b1[K1,N] in one split-K launch; None
// (nothing written) when the K-split plan does not fit the two buffers.
c10::optional<torch::Tensor> gemm_tn2(torch::Tensor a0, torch::Tensor b0, torch::Tensor a1, torch::Tensor b1,
                                      c10::optional<torch::Tensor> out, bool accumulate, int64_t variant) {
  TORCH_CHECK(variant == 0 || variant == 3, "gemm_tn2: variant 0 (v4) or 3 (v3)");
  for (auto* t : {&a0, &b0, &a1, &b1}) {
    check_rowmajor(*t, "gemm_tn2 operand");
    TORCH_CHECK(t->scalar_type() == torch::kBFloat16 && t->stride(0) % 8 == 0, "gemm_tn2: bf16, row stride % 8");
  }
  const int64_t K0 = a0.size(0), K1 = a1.size(0), M = a0.size(1), N = b0.size(1);
  TORCH_CHECK(b0.size(0) == K0 && b1.size(0) == K1 && a1.size(1) == M && b1.size(1) == N, "gemm_tn2: shape mismatch");
  TORCH_CHECK(M % 8 == 0 && N % 8 == 0, "gemm_tn2: M and N must be multiples of 8");
  TORCH_CHECK(a1.device() == a0.device() && b0.device() == a0.device() && b1.device() == a0.device(),
              "gemm_tn2: one device");
  const at::DeviceGuard g(a0.device());
  torch::Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    TORCH_CHECK(c.scalar_type() == torch::kFloat32 && c.is_contiguous() && c.size(0) == M && c.size(1) == N,
                "gemm_tn2: out must be contiguous fp32 [M,N]");
  } else {
    c = torch::empty({M, N}, a0.options().dtype(torch::kFloat32));
    accumulate = false;
  }
  if (M == 0 || N == 0 || K0 == 0 || K1 == 0) return c10::nullopt;
  const long long wsn = dpfs_gemm_tn2_ws((int)M, (int)N, (int)K0, (int)K1);
  if (wsn <= 0) return c10::nullopt;
  auto ws = torch::empty({wsn}, c.options());
  const int ok = dpfs_gemm_tn2(a0.data_ptr(), b0.data_ptr(), a1.data_ptr(), b1.data_ptr(), c.data_ptr<float>(),
                               ws.data_ptr<float>(), (int)M, (int)N, (int)K0, (int)K1, (int)a0.stride(0),
                               (int)b0.stride(0), (int)a1.stride(0), (int)b1.stride(0), accumulate ? 1 : 0,
                               (int)variant, stream());
  if (!ok) return c10::nullopt;
  return c;
}

torch::Tensor bias_grad(torch::Tensor dy) {
  check_rowmajor(dy, "dy");
  TORCH_CHECK(dy.is_contiguous(), "bias_grad: dy must be contiguous");
  const int64_t M = dy.size(0), N = dy.size(1);
  const int vec = dcode(dy) == 1 ? 8 : 4;
  TORCH_CHECK(N % vec == 0, "bias_grad: N must be a multiple of ", vec);
  const at::DeviceGuard g(dy.device());
  auto out = torch::empty({N}, dy.options().dtype(torch::kFloat32));
  if (M == 0) return out.zero_();
  auto ws = torch::empty({(int64_t)dpfs_colsum_ws((int)M, (int)N)}, out.options());
  dpfs_bias_grad(dcode(dy), dy.data_ptr(), out.data_ptr<float>(), ws.data_ptr<float>(), (int)M, (int)N, stream());
  return out;
}

torch::Tensor add_bias_(torch::Tensor y, torch::Tensor bias) {
  check_rowmajor(y, "y");
  TORCH_CHECK(y.is_contiguous(), "add_bias_: y must be contiguous");
  const int64_t M = y.size(0), N = y.size(1);
  const int vec = dcode(y) == 1 ? 8 : 4;
  TORCH_CHECK(N % vec == 0, "add_bias_: N must be a multiple of ", vec);
  const float* bp = opt_f32(bias, N, "bias");
  const at::DeviceGuard g(y.device());
  if (M) dpfs_bias_residual(dcode(y), y.data_ptr(), bp, nullptr, y.data_ptr(), (int)M, (int)N, stream());
  return y;
}

// out = residual + y (+ bias)
torch::Tensor bias_residual(torch::Tensor y, c10::optional<torch::Tensor> bias, torch::Tensor residual) {
  check_rowmajor(y, "y");
  TORCH_CHECK(y.is_contiguous() && residual.is_contiguous() && residual.sizes() == y.sizes() &&
                  residual.scalar_type() == y.scalar_type(),
              "bias_residual: y and residual must be contiguous, same shape/dtype");
  const int64_t M = y.size(0), N = y.size(1);
  const int vec = dcode(y) == 1 ? 8 : 4;
  TORCH_CHECK(N % vec == 0, "bias_residual: N must be a multiple of ", vec);
  const at::DeviceGuard g(y.device());
  auto out = torch::empty_like(y);
  if (M) dpfs_bias_residual(dcode(y), y.data_ptr(), opt_f32(bias, N, "bias"), residual.data_ptr(), out.data_ptr(),
                            (int)M, (int)N, stream());
  return out;
}

// ------------------------------------------------------------------------------- norms --
int check_norm_x(const torch::Tensor& x, const torch::Tensor& w) {
  check_rowmajor(x, "x");
  TORCH_CHECK(x.is_contiguous(), "norm: x must be contiguous");
  const int dt = dcode(x);
  const int64_t D = x.size(1);
  TORCH_CHECK(D % (dt == 1 ? 8 : 4) == 0 && D <= 32 * 64 * (dt == 1 ? 8 : 4), "norm: unsupported hidden size ", D);
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == torch::kFloat32 && w.is_contiguous() && w.numel() == D,
              "norm: weight must be contiguous fp32 [D]");
  return dt;
}

std::vector<torch::Tensor> rmsnorm_fwd(torch::Tensor x, torch::Tensor w, double eps) {
  const int dt = check_norm_x(x, w);
  const at::DeviceGuard g(x.device());
  const int64_t M = x.size(0), D = x.size(1);
  auto y = torch::empty_like(x);
  auto rstd = torch::empty({M}, x.options().dtype(torch::kFloat32));
  if (M) dpfs_rmsnorm_fwd(dt, x.data_ptr(), w.data_ptr<float>(), y.data_ptr(), rstd.data_ptr<float>(), (int)M, (int)D,
                          (float)eps, stream());
  return {y, rstd};
}

// (x = y + bias + res, RMSNorm(x), rstd) in one pass: the residual epilogue of a row-parallel
// projection fused into the next norm.
std::vector<torch::Tensor> add_rmsnorm_fwd(torch::Tensor y, c10::optional<torch::Tensor> bias, torch::Tensor res,
                                           torch::Tensor w, double eps) {
  const int dt = check_norm_x(res, w);
  TORCH_CHECK(y.sizes() == res.sizes() && y.is_contiguous() && y.scalar_type() == res.scalar_type(),
              "add_rmsnorm_fwd: y must match res");
  const at::DeviceGuard g(res.device());
  const int64_t M = res.size(0), D = res.size(1);
  const float* bp = opt_f32(bias, D, "bias");
  auto x = torch::empty_like(res);
  auto h = torch::empty_like(res);
  auto rstd = torch::empty({M}, res.options().dtype(torch::kFloat32));
  if (M)
    dpfs_add_rmsnorm_fwd(dt, y.data_ptr(), bp, res.data_ptr(), w.data_ptr<float>(), x.data_ptr(), h.data_ptr(),
                         rstd.data_ptr<float>(), (int)M, (int)D, (float)eps, stream());
  return {x, h, rstd};
}

static float* dbias_out(const c10::optional<torch::Tensor>& db, int64_t n, const char* what) {
  if (!db.has_value() || !db->defined()) return nullptr;
  TORCH_CHECK(db->is_cuda() && db->scalar_type() == torch::kFloat32 && db->is_contiguous() && db->numel() == n, what,
              ": dbias must be contiguous fp32 [", n, "]");
  return db->data_ptr<float>();
}

// dx = RMSNorm'(dy) (+ dres); with `dbias` also the column sums of dx (the bias grad of the
// projection whose output gradient dx is), from the same pass.
std::vector<torch::Tensor> rmsnorm_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor w, torch::Tensor rstd,
                                       c10::optional<torch::Tensor> dres, c10::optional<torch::Tensor> dbias,
                                       c10::optional<torch::Tensor> dw_out) {
  const int dt = check_norm_x(x, w);
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.is_contiguous() && dy.scalar_type() == x.scalar_type(), "rmsnorm_bwd: dy");
  const void* rp = nullptr;
  if (dres.has_value() && dres->defined()) {
    TORCH_CHECK(dres->sizes() == x.sizes() && dres->is_contiguous() && dres->scalar_type() == x.scalar_type(),
                "rmsnorm_bwd: dres must match x");
    rp = dres->data_ptr();
  }
  const at::DeviceGuard g(x.device());
  const int64_t M = x.size(0), D = x.size(1);
  float* db = dbias_out(dbias, x.size(1), "rmsnorm_bwd");
  auto dx = torch::empty_like(x);
  torch::Tensor dw;
  if (dw_out.has_value() && dw_out->defined()) {   // the weight gradient straight into its slot
    dw = *dw_out;
    TORCH_CHECK(dw.scalar_type() == torch::kFloat32 && dw.is_contiguous() && dw.numel() == D &&
                    dw.device() == x.device(),
                "rmsnorm_bwd: dw_out must be contiguous fp32 [D] on the device of x");
  } else {
    dw = torch::empty({D}, w.options());
  }
  if (M == 0) {
    if (db) dbias->zero_();
    return {dx, dw.zero_()};
  }
  const int mode = db ? 2 : 0;
  const int G = dpfs_norm_bwd_grid((int)M);
  auto ws = torch::empty({(int64_t)dpfs_norm_bwd_ws(mode, (int)M, (int)D)}, w.options());
  float* pw = ws.data_ptr<float>();
  dpfs_norm_bwd(mode, dt, dy.data_ptr(), x.data_ptr(), w.data_ptr<float>(), nullptr, rstd.data_ptr<float>(), rp,
                dx.data_ptr(), dw.data_ptr<float>(), db, pw, db ? pw + (int64_t)G * D : nullptr, (int)M, (int)D,
                stream());
  return {dx, dw};
}

std::vector<torch::Tensor> layernorm_fwd(torch::Tensor x, torch::Tensor w, torch::Tensor b, double eps) {
  const int dt = check_norm_x(x, w);
  TORCH_CHECK(b.is_cuda() && b.scalar_type() == torch::kFloat32 && b.numel() == x.size(1), "layernorm: bias");
  const at::DeviceGuard g(x.device());
  const int64_t M = x.size(0), D = x.size(1);
  auto y = torch::empty_like(x);
  auto mean = torch::empty({M}, x.options().dtype(torch::kFloat32));
  auto rstd = torch::empty({M}, x.options().dtype(torch::kFloat32));
  if (M) dpfs_layernorm_fwd(dt, x.data_ptr(), w.data_ptr<float>(), b.data_ptr<float>(), y.data_ptr(),
                            mean.data_ptr<float>(), rstd.data_ptr<float>(), (int)M, (int)D, (float)eps, stream());
  return {y, mean, rstd};
}

std::vector<torch::Tensor> layernorm_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor w, torch::Tensor mean,
                                         torch::Tensor rstd) {
  const int dt = check_norm_x(x, w);
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.is_contiguous() && dy.scalar_type() == x.scalar_type(),
              "layernorm_bwd: dy");
  const at::DeviceGuard g(x.device());
  const int64_t M = x.size(0), D = x.size(1);
  auto dx = torch::empty_like(x);
  auto dw = torch::empty({D}, w.options());
  auto db = torch::empty({D}, w.options());
  if (M == 0) return {dx, dw.zero_(), db.zero_()};
  const int64_t G = dpfs_norm_bwd_grid((int)M);
  auto ws = torch::empty({(int64_t)dpfs_norm_bwd_ws(1, (int)M, (int)D)}, w.options());
  dpfs_norm_bwd(1, dt, dy.data_ptr(), x.data_ptr(), w.data_ptr<float>(), mean.data_ptr<float>(),
                rstd.data_ptr<float>(), nullptr, dx.data_ptr(), dw.data_ptr<float>(), db.data_ptr<float>(),
                ws.data_ptr<float>(), ws.data_ptr<float>() + G * D, (int)M, (int)D, stream());
  return {dx, dw, db};
}

// ------------------------------------------------------------------------ elementwise --
// h = silu(gate) * up; `perm`: gu in the interleaved layout of the fused gate|up epilogue.
torch::Tensor swiglu_fwd(torch::Tensor gu, bool perm) {
  check_rowmajor(gu, "gu");
  TORCH_CHECK(gu.is_contiguous(), "swiglu: gu must be contiguous");
  const int dt = dcode(gu);
  const int64_t M = gu.size(0), F = gu.size(1) / 2;
  TORCH_CHECK(gu.size(1) % 2 == 0 && F % (dt == 1 ? 8 : 4) == 0, "swiglu: F must be a multiple of the vector width");
  TORCH_CHECK(!perm || F % 64 == 0, "swiglu: the interleaved layout needs F % 64 == 0");
  const at::DeviceGuard g(gu.device());
  auto h = torch::empty({M, F}, gu.options());
  if (M) dpfs_swiglu_fwd(dt, gu.data_ptr(), h.data_ptr(), (int)M, (int)F, perm ? 1 : 0, stream());
  return h;
}

// Gate|up projection with SwiGLU in the GEMM epilogue: w / bias in the natural [gate | up]
// layout, read with the rows interleaved in 64-row blocks (reference.gu_perm).  Returns
// [gu (interleaved), h] or [] where the fused kernel does not apply (the caller runs the GEMM
// on the interleaved weight + swiglu_fwd(perm)).
std::vector<torch::Tensor> gemm_nt_swiglu(torch::Tensor a, torch::Tensor b, c10::optional<torch::Tensor> bias) {
  check_rowmajor(a, "a");
  check_rowmajor(b, "b");
  TORCH_CHECK(a.scalar_type() == torch::kBFloat16 && b.scalar_type() == torch::kBFloat16,
              "gemm_nt_swiglu: bf16 operands");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K, "gemm_nt_swiglu: K mismatch");
  const at::DeviceGuard g(a.device());
  auto span = [](const torch::Tensor& t) -> long long {
    return t.size(0) > 0 ? ((t.size(0) - 1) * t.stride(0) + t.size(1)) * 2 : 0;
  };
  if (M == 0 || N % 128 || K % 64 || a.stride(0) % 8 || b.stride(0) % 8 || span(a) >= (1ll << 32) - 16 ||
      span(b) >= (1ll << 32) - 16)
    return {};
  auto c = torch::empty({M, N}, a.options());
  auto h = torch::empty({M, N / 2}, a.options());
  if (!dpfs_gemm4_nt_swiglu(a.data_ptr(), b.data_ptr(), c.data_ptr(), opt_f32(bias, N, "bias"), h.data_ptr(), (int)M,
                            (int)N, (int)K, (int)a.stride(0), (int)b.stride(0), (int)N, (int)(N / 2),
                            (unsigned)span(a), (unsigned)span(b), stream()))
    return {};
  return {c, h};
}


// dgu = SwiGLU'(gu) * dh; with `dbias` the gate|up bias gradient (column sums of dgu) is
// written there by the same pass.
torch::Tensor swiglu_bwd(torch::Tensor dh, torch::Tensor gu, c10::optional<torch::Tensor> dbias, bool perm) {
  check_rowmajor(gu, "gu");
  const int dt = dcode(gu);
  const int64_t M = gu.size(0), F = gu.size(1) / 2;
  TORCH_CHECK(dh.is_contiguous() && dh.size(0) == M && dh.size(1) == F && dh.scalar_type() == gu.scalar_type(),
              "swiglu_bwd: dh");
  TORCH_CHECK(F % (dt == 1 ? 8 : 4) == 0, "swiglu: F must be a multiple of the vector width");
  TORCH_CHECK(!perm || F % 64 == 0, "swiglu: the interleaved layout needs F % 64 == 0");
  const at::DeviceGuard g(gu.device());
  auto dgu = torch::empty_like(gu);
  float* db = dbias_out(dbias, 2 * F, "swiglu_bwd");
  if (db && M == 0) dbias->zero_();
  if (M == 0) return dgu;
  if (db) {
    TORCH_CHECK(gu.is_contiguous(), "swiglu_bwd: gu must be contiguous");
    const long long wsn = dpfs_swiglu_bwd_dbias_ws((int)M, (int)F);
    auto ws = torch::empty({std::max<long long>(wsn, 1)}, gu.options().dtype(torch::kFloat32));
    dpfs_swiglu_bwd_dbias(dt, dh.data_ptr(), gu.data_ptr(), dgu.data_ptr(), db, ws.data_ptr<float>(), (int)M, (int)F,
                          perm ? 1 : 0, stream());
  } else {
    dpfs_swiglu_bwd(dt, dh.data_ptr(), gu.data_ptr(), dgu.data_ptr(), (int)M, (int)F, perm ? 1 : 0, stream());
  }
  return dgu;
}

// Down-projection data gradient with the SwiGLU backward in its epilogue: dgu = SwiGLU'(gu) *
// (dy w) in the natural [gate | up] layout without materialising dy w (gu interleaved when
// `perm`); with `dbias` also the gate|up bias gradient (column sums of dgu) from the same
// kernel's partials.  Returns [] where the fused kernel does not apply (the caller runs
// gemm_nn + swiglu_bwd).
std::vector<torch::Tensor> gemm_nn_swiglu_bwd(torch::Tensor dy, torch::Tensor w, torch::Tensor gu,
                                              c10::optional<torch::Tensor> dbias, bool perm) {
  check_rowmajor(dy, "dy");
  check_rowmajor(w, "w");
  check_rowmajor(gu, "gu");
  TORCH_CHECK(dy.scalar_type() == torch::kBFloat16 && w.scalar_type() == torch::kBFloat16 &&
                  gu.scalar_type() == torch::kBFloat16, "gemm_nn_swiglu_bwd: bf16 operands");
  const int64_t M = dy.size(0), K = dy.size(1), F = w.size(1);
  TORCH_CHECK(w.size(0) == K && gu.size(0) == M && gu.size(1) == 2 * F, "gemm_nn_swiglu_bwd: shapes");
  const at::DeviceGuard g(dy.device());
  auto span = [](const torch::Tensor& t) -> long long {
    return t.size(0) > 0 ? ((t.size(0) - 1) * t.stride(0) + t.size(1)) * 2 : 0;
  };
  if (M == 0 || F % 64 || K % 64 || dy.stride(0) % 8 || w.stride(0) % 8 || gu.stride(0) % 8 ||
      span(dy) >= (1ll << 32) - 16 || span(w) >= (1ll << 32) - 16)
    return {};
  float* db = dbias_out(dbias, 2 * F, "gemm_nn_swiglu_bwd");
  auto dgu = torch::empty({M, 2 * F}, gu.options());
  const int64_t prow = 2 * ((M + 255) / 256);
  torch::Tensor part;
  if (db) part = torch::empty({prow, 2 * F}, gu.options().dtype(torch::kFloat32));
  if (!dpfs_gemm4_nn_swiglu_bwd(dy.data_ptr(), w.data_ptr(), gu.data_ptr(), dgu.data_ptr(),
                                db ? part.data_ptr<float>() : nullptr, (int)M, (int)F, (int)K, (int)dy.stride(0),
                                (int)w.stride(0), (int)gu.stride(0), (int)(2 * F), perm ? 1 : 0, (unsigned)span(dy),
                                (unsigned)span(w), stream()))
    return {};
  if (db) dpfs_colsum_rows_small(part.data_ptr<float>(), db, (int)prow, (int)(2 * F), stream());
  return {dgu};
}

torch::Tensor rope_(torch::Tensor qkv, torch::Tensor positions, torch::Tensor table, int64_t n_rot_heads,
                    int64_t head_dim, bool inverse) {
  check_rowmajor(qkv, "qkv");
  TORCH_CHECK(positions.is_cuda() && positions.scalar_type() == torch::kInt64 && positions.is_contiguous() &&
                  positions.numel() == qkv.size(0),
              "rope: positions must be contiguous int64 [M]");
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == torch::kFloat32 && table.is_contiguous() &&
                  table.dim() == 2 && table.size(1) == head_dim,
              "rope: table must be fp32 [maxlen, head_dim]");
  TORCH_CHECK(head_dim % 8 == 0, "rope: head_dim must be a multiple of 8");
  TORCH_CHECK(n_rot_heads * head_dim <= qkv.size(1), "rope: too many heads for the row");
  const at::DeviceGuard g(qkv.device());
  const int64_t M = qkv.size(0);
  if (M) dpfs_rope(dcode(qkv), qkv.data_ptr(), positions.data_ptr<int64_t>(), table.data_ptr<float>(), (int)M,
                   (int)qkv.stride(0), (int)n_rot_heads, (int)head_dim, inverse ? 1 : 0, stream());
  return qkv;
}

// ---------------------------------------------------------------------------- attention --
struct View4 {
  long long ld;
};

View4 check_bthd(const torch::Tensor& t, const char* name, int64_t B, int64_t T, int64_t H, int64_t hd) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16, name, " must be bf16");
  TORCH_CHECK(t.dim() == 4 && t.size(0) == B && t.size(1) == T && t.size(2) == H && t.size(3) == hd, name,
              " must be (B, T, H, hd)");
  TORCH_CHECK(t.stride(3) == 1 && t.stride(2) == hd && (B == 1 || t.stride(0) == T * t.stride(1)), name,
              " must be a (B*T, ld) row view with packed heads");
  TORCH_CHECK(t.stride(1) % 8 == 0, name, " token stride must be a multiple of 8");
  return {(long long)t.stride(1)};
}

std::vector<torch::Tensor> attn_fwd(torch::Tensor q, torch::Tensor k, torch::Tensor v, double scale, bool causal,
                                    int64_t impl) {
  const int64_t B = q.size(0), T = q.size(1), H = q.size(2), hd = q.size(3);
  TORCH_CHECK(dpfs_attn_supported_hd((int)hd), "attn: head_dim ", hd, " not supported (32/64/128)");
  auto vq = check_bthd(q, "q", B, T, H, hd), vk = check_bthd(k, "k", B, T, H, hd), vv = check_bthd(v, "v", B, T, H, hd);
  const at::DeviceGuard g(q.device());
  auto o = torch::empty({B, T, H, hd}, q.options());
  auto lse = torch::empty({B, H, T}, q.options().dtype(torch::kFloat32));
  if (B * T * H)
    dpfs_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), (int)B, (int)T,
                  (int)H, (int)hd, vq.ld, vk.ld, vv.ld, H * hd, (float)scale, causal ? 1 : 0, (int)impl, stream());
  return {o, lse};
}

// With dbias (fp32 [3 * H * hd], the packed QKV projection's bias layout) the q / k / v bias
// gradient (column sums of the stored dq / dk / dv) comes out of the same kernels; returns
// whether it did (false: another dK/dV variant is selected, dbias untouched).
bool attn_bwd(torch::Tensor dout, torch::Tensor q, torch::Tensor k, torch::Tensor v, torch::Tensor o,
              torch::Tensor lse, double scale, bool causal, torch::Tensor dq, torch::Tensor dk, torch::Tensor dv,
              c10::optional<torch::Tensor> rope_pos, c10::optional<torch::Tensor> rope_tab,
              c10::optional<torch::Tensor> dbias, int64_t impl) {
  const int64_t B = q.size(0), T = q.size(1), H = q.size(2), hd = q.size(3);
  TORCH_CHECK(dpfs_attn_supported_hd((int)hd), "attn: head_dim not supported");
  auto vq = check_bthd(q, "q", B, T, H, hd), vk = check_bthd(k, "k", B, T, H, hd), vv = check_bthd(v, "v", B, T, H, hd);
  auto vdo = check_bthd(dout, "dout", B, T, H, hd), vo = check_bthd(o, "o", B, T, H, hd);
  auto vdq = check_bthd(dq, "dq", B, T, H, hd), vdk = check_bthd(dk, "dk", B, T, H, hd),
       vdv = check_bthd(dv, "dv", B, T, H, hd);
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == torch::kFloat32 && lse.is_contiguous() && lse.numel() == B * H * T,
              "attn_bwd: lse must be contiguous fp32 (B, H, T)");
  const at::DeviceGuard g(q.device());
  float* db = nullptr;
  if (dbias.has_value() && dbias->defined()) {
    TORCH_CHECK(dbias->is_cuda() && dbias->scalar_type() == torch::kFloat32 && dbias->is_contiguous() &&
                    dbias->numel() == 3 * H * hd,
                "attn_bwd: dbias must be contiguous fp32 [3 * H * hd]");
    db = dbias->data_ptr<float>();
  }
  if (B * T * H == 0) {
    if (db) dbias->zero_();
    return db != nullptr;
  }
  const int64_t* rp = nullptr;
  const float* rt = nullptr;
  if (rope_pos.has_value() && rope_pos->defined()) {
    TORCH_CHECK(rope_pos->scalar_type() == torch::kInt64 && rope_pos->is_contiguous() && rope_pos->numel() == B * T,
                "attn_bwd: rope_pos must be contiguous int64 [B*T]");
    TORCH_CHECK(rope_tab.has_value() && rope_tab->scalar_type() == torch::kFloat32 && rope_tab->is_contiguous() &&
                    rope_tab->dim() == 2 && rope_tab->size(1) == hd,
                "attn_bwd: rope_tab must be contiguous fp32 [maxlen, hd]");
    rp = rope_pos->data_ptr<int64_t>();
    rt = rope_tab->data_ptr<float>();
  }
  auto delta = torch::empty({2, B, H, T}, lse.options());   // -delta | -lse/scale
  if (impl == 6 && dpfs_attn_fused_ws((int)B, (int)T, (int)H, (int)hd) > 0) {
    // fused backward (head_dim 64): fp32 dQ partials per (b, h, 256-key block, 64-query tile)
    auto dqp = torch::empty({dpfs_attn_fused_ws((int)B, (int)T, (int)H, (int)hd)}, lse.options());
    torch::Tensor fb;
    if (db) fb = torch::empty({dpfs_attn_fused_bias_ws((int)B, (int)T, (int)H, (int)hd)}, lse.options());
    return dpfs_attn_bwd_fused(dout.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                               lse.data_ptr<float>(), delta.data_ptr<float>(), dqp.data_ptr<float>(), dq.data_ptr(),
                               dk.data_ptr(), dv.data_ptr(), (int)B, (int)T, (int)H, (int)hd, vdo.ld, vq.ld, vk.ld,
                               vv.ld, vo.ld, vdq.ld, vdk.ld, vdv.ld, (float)scale, causal ? 1 : 0, rp, rt, stream(), db,
                               db ? fb.data_ptr<float>() : nullptr) > 0;
  }
  torch::Tensor bws;
  if (db) bws = torch::empty({dpfs_attn_bias_ws((int)B, (int)T, (int)H, (int)hd)}, lse.options());
  return dpfs_attn_bwd(dout.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(),
                       delta.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), (int)B, (int)T, (int)H,
                       (int)hd, vdo.ld, vq.ld, vk.ld, vv.ld, vo.ld, vdq.ld, vdk.ld, vdv.ld, (float)scale, causal ? 1 : 0,
                       rp, rt, stream(), db, db ? bws.data_ptr<float>() : nullptr, (int)impl) != 0;
}

// ----------------------------------------------------------------------- fp32 path --
// The reference's default (fp32) training on the device: fp32-input MFMA GEMMs and flash
// attention (csrc/kernels/fp32.hip).  layout 0 = NT: c[M,N] = a[M,K] b[N,K]^T (+ bias);
// 1 = NN: a[M,K] b[K,N]; 2 = TN: a[K,M]^T b[K,N] (+= into out with accumulate).
torch::Tensor gemm_f32(torch::Tensor a, torch::Tensor b, int64_t layout, c10::optional<torch::Tensor> bias,
                       c10::optional<torch::Tensor> out, bool accumulate) {
  check_cuda(a, "a");
  check_cuda(b, "b");
  const bool in16 = a.scalar_type() == torch::kBFloat16;
  TORCH_CHECK((a.scalar_type() == torch::kFloat32 || in16) && b.scalar_type() == a.scalar_type(),
              "gemm_f32: fp32 or bf16 operands (both alike)");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.stride(1) == 1 && b.stride(1) == 1, "gemm_f32: row-major 2-D operands");
  TORCH_CHECK(layout >= 0 && layout <= 2, "gemm_f32: layout 0 / 1 / 2");
  const int64_t M = layout == 2 ? a.size(1) : a.size(0), K = layout == 2 ? a.size(0) : a.size(1);
  const int64_t N = layout == 0 ? b.size(0) : b.size(1);
  TORCH_CHECK((layout == 0 ? b.size(1) : b.size(0)) == K, "gemm_f32: inner dimensions differ");
  const at::DeviceGuard g(a.device());
  torch::Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    TORCH_CHECK((c.scalar_type() == torch::kFloat32 || c.scalar_type() == torch::kBFloat16) && c.dim() == 2 &&
                    c.size(0) == M && c.size(1) == N && c.stride(1) == 1, "gemm_f32: out fp32 / bf16 [M, N] row-major");
  } else {
    // the bf16 API's output dtypes: a.dtype for NT / NN, fp32 for TN (weight gradients)
    c = torch::empty({M, N}, a.options().dtype(layout == 2 ? torch::kFloat32 : a.scalar_type()));
    accumulate = false;
  }
  TORCH_CHECK(in16 || c.scalar_type() == torch::kFloat32, "gemm_f32: fp32 operands give an fp32 output");
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->is_contiguous() && bias->numel() == N,
                "gemm_f32: bias fp32 [N]");
    bp = bias->data_ptr<float>();
  }
  if (M && N) {
    if (K == 0) {
      if (!accumulate) c.zero_();
      if (bp) c.add_(*bias);
    } else {
      const int sp = dpfs_gemm_f32_splits((int)M, (int)N, (int)K);   // K-split slabs (weight gradients)
      torch::Tensor ws;
      if (sp > 1) ws = torch::empty({(int64_t)sp * M * N}, a.options().dtype(torch::kFloat32));
      dpfs_gemm_f32((int)layout, a.data_ptr(), b.data_ptr(), c.data_ptr(), bp, (int)M, (int)N, (int)K, a.stride(0),
                    b.stride(0), c.stride(0), accumulate ? 1 : 0, sp > 1 ? ws.data_ptr<float>() : nullptr,
                    in16 ? 1 : 0, c.scalar_type() == torch::kBFloat16 ? 1 : 0, stream());
    }
  }
  return c;
}

View4 check_bthd_f32(const torch::Tensor& t, const char* name, int64_t B, int64_t T, int64_t H, int64_t hd) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be fp32");
  TORCH_CHECK(t.dim() == 4 && t.size(0) == B && t.size(1) == T && t.size(2) == H && t.size(3) == hd, name,
              " must be (B, T, H, hd)");
  TORCH_CHECK(t.stride(3) == 1 && t.stride(2) == hd && (B == 1 || t.stride(0) == T * t.stride(1)), name,
              " must be a (B*T, ld) row view with packed heads");
  TORCH_CHECK(t.stride(1) % 4 == 0 && (reinterpret_cast<uintptr_t>(t.data_ptr()) % 16) == 0, name,
              " token stride must be a multiple of 4 floats (16-byte rows)");
  return {(long long)t.stride(1)};
}

std::vector<torch::Tensor> attn_fwd_f32(torch::Tensor q, torch::Tensor k, torch::Tensor v, double scale, bool causal) {
  const int64_t B = q.size(0), T = q.size(1), H = q.size(2), hd = q.size(3);
  TORCH_CHECK(dpfs_attn_f32_supported_hd((int)hd), "attn_fwd_f32: head_dim ", hd, " not supported (32/64/128)");
  auto vq = check_bthd_f32(q, "q", B, T, H, hd), vk = check_bthd_f32(k, "k", B, T, H, hd),
       vv = check_bthd_f32(v, "v", B, T, H, hd);
  const at::DeviceGuard g(q.device());
  auto o = torch::empty({B, T, H, hd}, q.options());
  auto lse = torch::empty({B, H, T}, q.options());
  if (B * T * H)
    dpfs_attn_fwd_f32(q.data_ptr<float>(), k.data_ptr<float>(), v.data_ptr<float>(), o.data_ptr<float>(),
                      lse.data_ptr<float>(), (int)B, (int)T, (int)H, (int)hd, vq.ld, vk.ld, vv.ld, H * hd,
                      (float)scale, causal ? 1 : 0, stream());
  return {o, lse};
}

bool attn_bwd_f32(torch::Tensor dout, torch::Tensor q, torch::Tensor k, torch::Tensor v, torch::Tensor o,
                  torch::Tensor lse, double scale, bool causal, torch::Tensor dq, torch::Tensor dk, torch::Tensor dv,
                  c10::optional<torch::Tensor> rope_pos, c10::optional<torch::Tensor> rope_tab,
                  c10::optional<torch::Tensor> dbias) {
  const int64_t B = q.size(0), T = q.size(1), H = q.size(2), hd = q.size(3);
  TORCH_CHECK(dpfs_attn_f32_supported_hd((int)hd), "attn_bwd_f32: head_dim not supported");
  auto vq = check_bthd_f32(q, "q", B, T, H, hd), vk = check_bthd_f32(k, "k", B, T, H, hd),
       vv = check_bthd_f32(v, "v", B, T, H, hd);
  auto vdo = check_bthd_f32(dout, "dout", B, T, H, hd), vo = check_bthd_f32(o, "o", B, T, H, hd);
  auto vdq = check_bthd_f32(dq, "dq", B, T, H, hd), vdk = check_bthd_f32(dk, "dk", B, T, H, hd),
       vdv = check_bthd_f32(dv, "dv", B, T, H, hd);
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == torch::kFloat32 && lse.is_contiguous() && lse.numel() == B * H * T,
              "attn_bwd_f32: lse must be contiguous fp32 (B, H, T)");
  const at::DeviceGuard g(q.device());
  float* db = nullptr;
  if (dbias.has_value() && dbias->defined()) {
    TORCH_CHECK(dbias->is_cuda() && dbias->scalar_type() == torch::kFloat32 && dbias->is_contiguous() &&
                    dbias->numel() == 3 * H * hd, "attn_bwd_f32: dbias must be contiguous fp32 [3 * H * hd]");
    db = dbias->data_ptr<float>();
  }
  if (B * T * H == 0) {
    if (db) dbias->zero_();
    return db != nullptr;
  }
  const int64_t* rp = nullptr;
  const float* rt = nullptr;
  if (rope_pos.has_value() && rope_pos->defined()) {
    TORCH_CHECK(rope_pos->scalar_type() == torch::kInt64 && rope_pos->is_contiguous() && rope_pos->numel() == B * T,
                "attn_bwd_f32: rope_pos must be contiguous int64 [B*T]");
    TORCH_CHECK(rope_tab.has_value() && rope_tab->scalar_type() == torch::kFloat32 && rope_tab->is_contiguous() &&
                    rope_tab->dim() == 2 && rope_tab->size(1) == hd, "attn_bwd_f32: rope_tab fp32 [maxlen, hd]");
    rp = rope_pos->data_ptr<int64_t>();
    rt = rope_tab->data_ptr<float>();
  }
  auto ws = torch::empty({dpfs_attn_bwd_f32_ws((int)B, (int)T, (int)H, (int)hd, db ? 1 : 0)}, lse.options());
  return dpfs_attn_bwd_f32(dout.data_ptr<float>(), q.data_ptr<float>(), k.data_ptr<float>(), v.data_ptr<float>(),
                           o.data_ptr<float>(), lse.data_ptr<float>(), ws.data_ptr<float>(), dq.data_ptr<float>(),
                           dk.data_ptr<float>(), dv.data_ptr<float>(), (int)B, (int)T, (int)H, (int)hd, vdo.ld, vq.ld,
                           vk.ld, vv.ld, vo.ld, vdq.ld, vdk.ld, vdv.ld, (float)scale, causal ? 1 : 0, rp, rt, db,
                           stream()) != 0;
}

// ------------------------------------------------------------------- embedding / CE --
torch::Tensor embedding_fwd(torch::Tensor ids, torch::Tensor weight, int64_t vocab_start, py::object out_dtype) {
  check_cuda(ids, "ids");
  check_cuda(weight, "weight");
  TORCH_CHECK(ids.scalar_type() == torch::kInt64 && ids.is_contiguous() && ids.dim() == 1, "embedding: ids int64 [M]");
  TORCH_CHECK(weight.scalar_type() == torch::kFloat32 && weight.is_contiguous() && weight.dim() == 2 &&
                  weight.size(1) % 4 == 0,
              "embedding: weight must be contiguous fp32 [V_local, D], D % 4 == 0");
  const auto odt = torch::python::detail::py_object_to_dtype(out_dtype);
  TORCH_CHECK(odt == torch::kBFloat16 || odt == torch::kFloat32, "embedding: out dtype bf16/fp32");
  const at::DeviceGuard g(ids.device());
  const int64_t M = ids.numel(), D = weight.size(1);
  auto out = torch::empty({M, D}, weight.options().dtype(odt));
  if (M) dpfs_embedding_fwd(odt == torch::kBFloat16 ? 1 : 0, ids.data_ptr<int64_t>(), weight.data_ptr<float>(),
                            out.data_ptr(), (int)M, (int)D, vocab_start, (int)weight.size(0), stream());
  return out;
}

// fp32 dW[v_local, D] of the masked embedding; with ``out`` the rows are ADDED to it (the
// engines' gradient arena: zeroed once per step, every chunk accumulates).
torch::Tensor embedding_bwd(torch::Tensor dout, torch::Tensor ids, int64_t v_local, int64_t vocab_start,
                            c10::optional<torch::Tensor> out) {
  check_rowmajor(dout, "dout");
  TORCH_CHECK(dout.is_contiguous(), "embedding_bwd: dout contiguous");
  TORCH_CHECK(ids.scalar_type() == torch::kInt64 && ids.is_contiguous() && ids.numel() == dout.size(0),
              "embedding_bwd: ids");
  const at::DeviceGuard g(dout.device());
  const int64_t M = dout.size(0), D = dout.size(1);
  torch::Tensor dw;
  if (out.has_value()) {
    dw = *out;
    TORCH_CHECK(dw.scalar_type() == torch::kFloat32 && dw.is_contiguous() && dw.dim() == 2 && dw.size(0) == v_local &&
                    dw.size(1) == D && dw.device() == dout.device(),
                "embedding_bwd: out must be contiguous fp32 [v_local, D] on the device of dout");
  } else {
    dw = torch::zeros({v_local, D}, dout.options().dtype(torch::kFloat32));
  }
  if (M) dpfs_embedding_bwd(dcode(dout), dout.data_ptr(), ids.data_ptr<int64_t>(), dw.data_ptr<float>(), (int)M,
                            (int)D, vocab_start, (int)v_local, stream());
  return dw;
}

// Deterministic embedding gradient (no atomics): the ids sorted (stable), each local vocab row's
// segment found by binary search, one wave per vocab row sums its rows in row order and WRITES
// dw (every row: no zero pass), or adds to it (`accumulate`).  D % 4 == 0 (else the atomic form).
// Stable order of the ids by local vocab row (ids outside [vocab_start, vocab_start + v_local)
// last) and each row's segment start: the deterministic embedding backward's index
// (embedding_bwd_sorted); a two-pass radix sort on our kernels (embedding_ce.hip).
std::vector<torch::Tensor> emb_sort(torch::Tensor ids, int64_t vocab_start, int64_t v_local) {
  check_cuda(ids, "ids");
  TORCH_CHECK(ids.scalar_type() == torch::kInt64 && ids.is_contiguous(), "emb_sort: ids int64 contiguous");
  TORCH_CHECK(v_local >= 0 && v_local < 65535, "emb_sort: the local vocab must be below 65535 rows");
  TORCH_CHECK(ids.numel() < (1LL << 31), "emb_sort: too many ids");
  const at::DeviceGuard g(ids.device());
  const int M = (int)ids.numel();
  auto ws = torch::empty({dpfs_emb_sort_ws(M)}, ids.options().dtype(torch::kInt32));
  auto perm = torch::empty({M}, ids.options());
  auto seg = torch::empty({v_local + 1}, ids.options());
  dpfs_emb_sort(ids.data_ptr<int64_t>(), M, vocab_start, (int)v_local, ws.data_ptr<int>(), perm.data_ptr<int64_t>(),
                seg.data_ptr<int64_t>(), stream());
  return {perm, seg};
}

torch::Tensor embedding_bwd_sorted(torch::Tensor dout, torch::Tensor ids, int64_t v_local, int64_t vocab_start,
                                   c10::optional<torch::Tensor> out, bool accumulate,
                                   c10::optional<torch::Tensor> perm_in, c10::optional<torch::Tensor> seg_in) {
  check_rowmajor(dout, "dout");
  TORCH_CHECK(dout.is_contiguous(), "embedding_bwd_sorted: dout contiguous");
  TORCH_CHECK(ids.scalar_type() == torch::kInt64 && ids.is_contiguous() && ids.numel() == dout.size(0),
              "embedding_bwd_sorted: ids");
  const at::DeviceGuard g(dout.device());
  const int64_t D = dout.size(1);
  torch::Tensor dw;
  if (out.has_value()) {
    dw = *out;
    TORCH_CHECK(dw.scalar_type() == torch::kFloat32 && dw.is_contiguous() && dw.dim() == 2 && dw.size(0) == v_local &&
                    dw.size(1) == D && dw.device() == dout.device(),
                "embedding_bwd_sorted: out must be contiguous fp32 [v_local, D] on the device of dout");
  } else {
    dw = torch::empty({v_local, D}, dout.options().dtype(torch::kFloat32));
    accumulate = false;
  }
  if (v_local == 0) return dw;
  if (D % 4) {   // (the atomic form needs a zeroed / accumulating output)
    if (!accumulate) dw.zero_();
    return embedding_bwd(dout, ids, v_local, vocab_start, dw);
  }
  torch::Tensor perm, seg;
  if (perm_in.has_value() && seg_in.has_value()) {   // sorted ahead (e.g. on a side stream in the forward)
    perm = *perm_in;
    seg = *seg_in;
    TORCH_CHECK(perm.scalar_type() == torch::kInt64 && perm.is_contiguous() && perm.numel() == ids.numel() &&
                    seg.scalar_type() == torch::kInt64 && seg.is_contiguous() && seg.numel() == v_local + 1,
                "embedding_bwd_sorted: perm [M] / seg [v_local + 1] int64");
  } else {
    auto ps = emb_sort(ids, vocab_start, v_local);
    perm = ps[0];
    seg = ps[1];
  }
  dpfs_embedding_bwd_seg(dcode(dout), dout.data_ptr(), perm.data_ptr<int64_t>(), seg.data_ptr<int64_t>(),
                         dw.data_ptr<float>(), (int)D, (int)v_local, accumulate ? 1 : 0, stream());
  return dw;
}

// Loss bookkeeping of the vocab-parallel CE from the gathered statistics (nsh, M, 3): per-row
// lse and validity (1.0 / 0.0), the running (loss sum, valid count) in acc[2] (overwritten when
// `first`), and with `last` the mean loss into `loss` (0-d) and max(count, 1) into acc[1].
std::vector<torch::Tensor> ce_finalize(torch::Tensor stats, torch::Tensor targets, int64_t ignore_index,
                                       torch::Tensor acc, torch::Tensor loss, bool first, bool last) {
  check_cuda(stats, "stats");
  TORCH_CHECK(stats.scalar_type() == torch::kFloat32 && stats.is_contiguous() && stats.dim() == 3 &&
                  stats.size(2) == 3, "ce_finalize: stats fp32 contiguous (nsh, M, 3)");
  const int64_t M = stats.size(1);
  TORCH_CHECK(targets.scalar_type() == torch::kInt64 && targets.is_contiguous() && targets.numel() == M,
              "ce_finalize: targets int64 [M]");
  TORCH_CHECK(acc.scalar_type() == torch::kFloat32 && acc.is_contiguous() && acc.numel() >= 2 &&
                  loss.scalar_type() == torch::kFloat32 && loss.numel() == 1 && loss.is_contiguous(),
              "ce_finalize: acc fp32 [>=2], loss fp32 scalar");
  const at::DeviceGuard g(stats.device());
  auto lse = torch::empty({M}, stats.options());
  auto valid = torch::empty({M}, stats.options());
  auto part = torch::empty({dpfs_ce_part_floats()}, stats.options());
  dpfs_ce_finalize(stats.data_ptr<float>(), targets.data_ptr<int64_t>(), ignore_index, lse.data_ptr<float>(),
                   valid.data_ptr<float>(), acc.data_ptr<float>(), loss.data_ptr<float>(), part.data_ptr<float>(),
                   (int)M, (int)stats.size(0), first ? 1 : 0, last ? 1 : 0, stream());
  return {lse, valid};
}

std::vector<torch::Tensor> ce_valid_scale(torch::Tensor targets, int64_t ignore_index) {
  check_cuda(targets, "targets");
  TORCH_CHECK(targets.scalar_type() == torch::kInt64 && targets.is_contiguous(), "ce_valid_scale: int64 targets");
  const at::DeviceGuard g(targets.device());
  const int64_t M = targets.numel();
  auto gs = torch::empty({M}, targets.options().dtype(torch::kFloat32));
  auto n = torch::empty({}, targets.options().dtype(torch::kFloat32));
  auto part = torch::empty({dpfs_ce_part_floats()}, targets.options().dtype(torch::kFloat32));
  dpfs_ce_valid_scale(targets.data_ptr<int64_t>(), ignore_index, gs.data_ptr<float>(), n.data_ptr<float>(),
                      part.data_ptr<float>(), (int)M, stream());
  return {gs, n};
}

torch::Tensor ce_grad_scale(torch::Tensor valid, torch::Tensor gloss, torch::Tensor n_valid) {
  check_cuda(valid, "valid");
  TORCH_CHECK(valid.scalar_type() == torch::kFloat32 && valid.is_contiguous(), "ce_grad_scale: fp32 valid [M]");
  TORCH_CHECK((gloss.scalar_type() == torch::kFloat32 || gloss.scalar_type() == torch::kBFloat16) && gloss.numel() == 1 &&
                  gloss.is_cuda(), "ce_grad_scale: gloss fp32 / bf16 scalar on the device");
  TORCH_CHECK(n_valid.scalar_type() == torch::kFloat32 && n_valid.numel() == 1 && n_valid.is_cuda(),
              "ce_grad_scale: n_valid fp32 scalar on the device");
  const at::DeviceGuard g(valid.device());
  auto gs = torch::empty_like(valid);
  auto gl = gloss.contiguous();
  auto nv = n_valid.contiguous();
  dpfs_ce_grad_scale(valid.data_ptr<float>(), gl.data_ptr(), gl.scalar_type() == torch::kBFloat16 ? 1 : 0,
                     nv.data_ptr<float>(), gs.data_ptr<float>(), (int)valid.numel(), stream());
  return gs;
}

torch::Tensor ce_fwd_stats(torch::Tensor logits, torch::Tensor targets, int64_t vocab_start, int64_t vocab_valid) {
  check_rowmajor(logits, "logits");
  TORCH_CHECK(logits.is_contiguous(), "ce: logits contiguous");
  TORCH_CHECK(targets.scalar_type() == torch::kInt64 && targets.is_contiguous() && targets.numel() == logits.size(0),
              "ce: targets int64 [M]");
  TORCH_CHECK(vocab_valid >= 0 && vocab_valid <= logits.size(1), "ce: vocab_valid out of range");
  const at::DeviceGuard g(logits.device());
  const int64_t M = logits.size(0), V = logits.size(1);
  auto stats = torch::empty({M, 3}, logits.options().dtype(torch::kFloat32));
  if (M) dpfs_ce_stats(dcode(logits), logits.data_ptr(), targets.data_ptr<int64_t>(), stats.data_ptr<float>(), (int)M,
                       (int)V, vocab_start, (int)vocab_valid, stream());
  return stats;
}

// Single-shard CE forward + backward in one pass (TP 1): returns the ce_fwd_stats rows and
// overwrites logits with (softmax - onehot) * gscale[row] (+ the bias gradient into dbias);
// None (nothing launched) where the one-pass kernel does not apply.
c10::optional<torch::Tensor> ce_fused(torch::Tensor logits, torch::Tensor targets, torch::Tensor gscale,
                                      int64_t vocab_start, int64_t vocab_valid, c10::optional<torch::Tensor> dbias) {
  check_rowmajor(logits, "logits");
  TORCH_CHECK(logits.is_contiguous(), "ce_fused: logits contiguous");
  const int64_t M = logits.size(0), V = logits.size(1);
  TORCH_CHECK(targets.scalar_type() == torch::kInt64 && targets.is_contiguous() && targets.numel() == M,
              "ce_fused: targets int64 [M]");
  TORCH_CHECK(gscale.scalar_type() == torch::kFloat32 && gscale.is_contiguous() && gscale.numel() == M,
              "ce_fused: gscale fp32 [M]");
  TORCH_CHECK(vocab_valid >= 0 && vocab_valid <= V, "ce_fused: vocab_valid out of range");
  TORCH_CHECK(M < (1ll << 31) / 3, "ce_fused: too many rows");
  const at::DeviceGuard g(logits.device());
  float* db = dbias_out(dbias, V, "ce_fused");
  auto stats = torch::empty({M, 3}, logits.options().dtype(torch::kFloat32));
  torch::Tensor ws;
  if (db) ws = torch::empty({std::max<long long>(dpfs_ce_fused_ws((int)M, (int)V), 1)}, stats.options());
  if (db && M == 0) dbias->zero_();
  const int ok = dpfs_ce_fused(dcode(logits), logits.data_ptr(), targets.data_ptr<int64_t>(), gscale.data_ptr<float>(),
                               stats.data_ptr<float>(), db, db ? ws.data_ptr<float>() : nullptr, (int)M, (int)V,
                               vocab_start, (int)vocab_valid, stream());
  if (!ok) return c10::nullopt;
  return stats;
}

torch::Tensor ce_bwd(torch::Tensor logits, torch::Tensor targets, torch::Tensor lse, torch::Tensor gscale,
                     int64_t vocab_start, int64_t vocab_valid, torch::Tensor out,
                     c10::optional<torch::Tensor> dbias) {
  check_rowmajor(logits, "logits");
  TORCH_CHECK(logits.is_contiguous() && out.is_contiguous() && out.sizes() == logits.sizes() &&
                  out.scalar_type() == logits.scalar_type(),
              "ce_bwd: out must match logits");
  const int64_t M = logits.size(0), V = logits.size(1);
  TORCH_CHECK(lse.scalar_type() == torch::kFloat32 && lse.numel() == M && gscale.scalar_type() == torch::kFloat32 &&
                  gscale.numel() == M && lse.is_contiguous() && gscale.is_contiguous(),
              "ce_bwd: lse/gscale fp32 [M]");
  const at::DeviceGuard g(logits.device());
  float* db = dbias_out(dbias, V, "ce_bwd");
  if (db && M == 0) dbias->zero_();
  if (M == 0) return out;
  if (db) {
    const long long wsn = dpfs_ce_bwd_dbias_ws(dcode(logits), (int)M, (int)V);
    auto ws = torch::empty({std::max<long long>(wsn, 1)}, lse.options());
    dpfs_ce_bwd_dbias(dcode(logits), logits.data_ptr(), targets.data_ptr<int64_t>(), lse.data_ptr<float>(),
                      gscale.data_ptr<float>(), out.data_ptr(), db, ws.data_ptr<float>(), (int)M, (int)V, vocab_start,
                      (int)vocab_valid, stream());
  } else {
    dpfs_ce_bwd(dcode(logits), logits.data_ptr(), targets.data_ptr<int64_t>(), lse.data_ptr<float>(),
                gscale.data_ptr<float>(), out.data_ptr(), (int)M, (int)V, vocab_start, (int)vocab_valid, stream());
  }
  return out;
}

// --------------------------------------------------------------------------------- Adam --
// Builds the device descriptor table for a fixed list of tensors (done once).
std::vector<torch::Tensor> adam_build(std::vector<torch::Tensor> params, std::vector<torch::Tensor> grads,
                                      std::vector<torch::Tensor> m, std::vector<torch::Tensor> v,
                                      std::vector<c10::optional<torch::Tensor>> shadows) {
  const size_t n = params.size();
  TORCH_CHECK(grads.size() == n && m.size() == n && v.size() == n && shadows.size() == n, "adam_build: list sizes");
  const int db = dpfs_adam_desc_bytes();
  TORCH_CHECK(db == 48, "unexpected AdamTensor layout");
  std::vector<int64_t> desc(n * 6);
  std::vector<int32_t> chunks;
  const int64_t C = dpfs_adam_chunk();
  for (size_t i = 0; i < n; ++i) {
    auto chk = [&](const torch::Tensor& t, const char* nm) {
      TORCH_CHECK(t.is_cuda() && t.scalar_type() == torch::kFloat32 && t.is_contiguous() &&
                      t.numel() == params[i].numel(),
                  "adam_build: ", nm, " must be contiguous fp32 matching the param");
    };
    chk(params[i], "param");
    chk(grads[i], "grad");
    chk(m[i], "exp_avg");
    chk(v[i], "exp_avg_sq");
    int64_t sh = 0;
    if (shadows[i].has_value() && shadows[i]->defined()) {
      TORCH_CHECK(shadows[i]->scalar_type() == torch::kBFloat16 && shadows[i]->is_contiguous() &&
                      shadows[i]->numel() == params[i].numel(),
                  "adam_build: shadow must be contiguous bf16");
      sh = (int64_t)shadows[i]->data_ptr();
    }
    desc[i * 6 + 0] = (int64_t)params[i].data_ptr();
    desc[i * 6 + 1] = (int64_t)grads[i].data_ptr();
    desc[i * 6 + 2] = (int64_t)m[i].data_ptr();
    desc[i * 6 + 3] = (int64_t)v[i].data_ptr();
    desc[i * 6 + 4] = sh;
    desc[i * 6 + 5] = params[i].numel();
    const int64_t nc = (params[i].numel() + C - 1) / C;
    for (int64_t c = 0; c < nc; ++c) {
      chunks.push_back((int32_t)i);
      chunks.push_back((int32_t)c);
    }
  }
  auto dev = params.empty() ? torch::Device(torch::kCUDA) : params[0].device();
  // Pinned staging + async copies: a pageable H2D copy would block the host until the GPU
  // has drained every queued kernel (the whole backward), idling the GPU while the host then
  // enqueues the optimizer and the next step.  The caching host allocator keeps the pinned
  // blocks alive until their copies have run.
  auto d = torch::from_blob(desc.data(), {(int64_t)desc.size()}, torch::kInt64).pin_memory().to(dev, true);
  auto c = torch::from_blob(chunks.data(), {(int64_t)chunks.size()}, torch::kInt32).pin_memory().to(dev, true);
  return {d, c};
}

// Rewrite the gradient pointers of a descriptor table built by adam_build (same params,
// same order; only the gradient tensors changed) without a host -> device copy.
void adam_patch_grads(torch::Tensor desc, std::vector<torch::Tensor> grads) {
  TORCH_CHECK(desc.is_cuda() && desc.scalar_type() == torch::kInt64 && desc.numel() == (int64_t)grads.size() * 6,
              "adam_patch_grads: descriptor table / grad list mismatch");
  std::vector<long long> ptrs(grads.size());
  for (size_t i = 0; i < grads.size(); ++i) {
    TORCH_CHECK(grads[i].is_cuda() && grads[i].scalar_type() == torch::kFloat32 && grads[i].is_contiguous(),
                "adam_patch_grads: grads must be contiguous fp32 on the device");
    ptrs[i] = (long long)grads[i].data_ptr();
  }
  const at::DeviceGuard g(desc.device());
  dpfs_adam_patch_grads(desc.data_ptr(), ptrs.data(), (int)ptrs.size(), stream());
}

void adam_step(torch::Tensor desc, torch::Tensor chunks, double lr, double b1, double b2, double eps, double wd,
               int64_t step, double gscale, c10::optional<torch::Tensor> dscale) {
  TORCH_CHECK(desc.is_cuda() && chunks.is_cuda(), "adam_step: tables must be on the device");
  const double bc1 = 1.0 - std::pow(b1, (double)step);
  const double bc2 = 1.0 - std::pow(b2, (double)step);
  const float* ds = nullptr;
  if (dscale.has_value() && dscale->defined()) {
    TORCH_CHECK(dscale->scalar_type() == torch::kFloat32 && dscale->numel() == 1, "adam_step: dscale fp32 scalar");
    ds = dscale->data_ptr<float>();
  }
  const at::DeviceGuard g(desc.device());
  dpfs_adam_step(desc.data_ptr(), chunks.data_ptr<int32_t>(), (int)(chunks.numel() / 2), (float)lr, (float)b1,
                 (float)b2, (float)eps, (float)wd, (float)bc1, (float)std::sqrt(bc2), (float)gscale, ds, stream());
}

torch::Tensor grad_sumsq(torch::Tensor desc, torch::Tensor chunks) {
  const at::DeviceGuard g(desc.device());
  const int n = (int)(chunks.numel() / 2);
  auto partial = torch::empty({n}, desc.options().dtype(torch::kFloat32));
  dpfs_grad_sumsq(desc.data_ptr(), chunks.data_ptr<int32_t>(), n, partial.data_ptr<float>(), stream());
  return partial.sum();
}

// ----------------------------------------------------------------------------- decode --
void check_cache(const torch::Tensor& c, const char* name) {
  check_cuda(c, name);
  TORCH_CHECK(c.dim() == 4 && c.is_contiguous() && c.scalar_type() == torch::kBFloat16, name,
              " must be a contiguous bf16 (B, T_max, H, hd) cache");
}

void check_len(const torch::Tensor& len) {
  check_cuda(len, "len");
  TORCH_CHECK(len.scalar_type() == torch::kInt32 && len.numel() == 1, "len must be a device int32 scalar");
}

// o[B, H*hd] = softmax(q k^T * scale) v over keys [0, *len] of the cache (one query per
// sequence and head).  q: [B, >= H*hd] rows (e.g. the q part of the packed qkv row).
torch::Tensor attn_decode(torch::Tensor q, torch::Tensor kc, torch::Tensor vc, torch::Tensor len, double scale) {
  check_rowmajor(q, "q");
  check_cache(kc, "k_cache");
  check_cache(vc, "v_cache");
  check_len(len);
  TORCH_CHECK(kc.sizes() == vc.sizes(), "k / v cache shapes differ");
  const int64_t B = kc.size(0), Tmax = kc.size(1), H = kc.size(2), hd = kc.size(3);
  TORCH_CHECK(hd == 32 || hd == 64 || hd == 128, "attn_decode: head_dim 32, 64 or 128");
  TORCH_CHECK(q.size(0) == B && q.size(1) >= H * hd && q.stride(0) % 8 == 0 && q.scalar_type() == torch::kBFloat16,
              "attn_decode: q rows");
  const at::DeviceGuard g(q.device());
  auto o = torch::empty({B, H * hd}, q.options());
  const int ns = dpfs_decode_nsplit((int)Tmax);
  auto part = torch::empty({B * H * ns * (hd + 2)}, q.options().dtype(torch::kFloat32));
  dpfs_attn_decode(q.data_ptr(), q.stride(0), kc.data_ptr(), vc.data_ptr(), len.data_ptr<int>(), o.data_ptr(), H * hd,
                   part.data_ptr<float>(), (int)B, (int)H, (int)hd, (int)Tmax, (float)scale, stream());
  return o;
}

// Write the k / v parts of the packed qkv rows [B, 3*H*hd] into the caches at row *len.
void kv_append(torch::Tensor qkv, torch::Tensor kc, torch::Tensor vc, torch::Tensor len) {
  check_rowmajor(qkv, "qkv");
  check_cache(kc, "k_cache");
  check_cache(vc, "v_cache");
  check_len(len);
  const int64_t B = kc.size(0), Tmax = kc.size(1), H = kc.size(2), hd = kc.size(3);
  TORCH_CHECK(qkv.size(0) == B && qkv.size(1) == 3 * H * hd && qkv.stride(0) % 8 == 0 &&
                  qkv.scalar_type() == torch::kBFloat16,
              "kv_append: qkv must be [B, 3*H*hd] bf16");
  const at::DeviceGuard g(qkv.device());
  const char* p = static_cast<const char*>(qkv.data_ptr());
  dpfs_kv_append(p + H * hd * 2, p + 2 * H * hd * 2, qkv.stride(0), kc.data_ptr(), vc.data_ptr(), len.data_ptr<int>(),
                 (int)B, (int)H, (int)hd, (int)Tmax, stream());
}

// y[M, N] = x[M, K] w[N, K]^T (+ bias) for M <= 16 (decode-step projections); with swiglu,
// x is the packed [M, 2K] gate|up output and the operand is silu(gate) * up.
bool gemv_nt_ok(torch::Tensor x, torch::Tensor w, bool swiglu) {
  if (!x.is_cuda() || x.dim() != 2 || w.dim() != 2 || x.scalar_type() != torch::kBFloat16 ||
      w.scalar_type() != torch::kBFloat16 || x.stride(1) != 1 || w.stride(1) != 1)
    return false;
  const int64_t K = w.size(1);
  if (x.size(1) != (swiglu ? 2 * K : K)) return false;
  if (reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 || reinterpret_cast<uintptr_t>(w.data_ptr()) % 16)
    return false;   // 16-byte operand loads
  return dpfs_gemv16_ok((int)x.size(0), (int)w.size(0), (int)K, x.stride(0), w.stride(0)) != 0;
}

torch::Tensor gemv_nt(torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> bias, bool swiglu) {
  TORCH_CHECK(gemv_nt_ok(x, w, swiglu), "gemv_nt: needs bf16 row-major x [M <= 16, K or 2K], w [N, K], K % 32 == 0");
  const int64_t M = x.size(0), N = w.size(0), K = w.size(1);
  const at::DeviceGuard g(x.device());
  auto y = torch::empty({M, N}, x.options());
  dpfs_gemv16(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), opt_f32(bias, N, "bias"), y.data_ptr(), N, (int)M,
              (int)N, (int)K, swiglu ? 1 : 0, stream());
  return y;
}

// rope_ on the q and k heads of the packed qkv rows + kv_append of the rotated k and v rows
// at *len, one kernel (decode step).
void rope_append(torch::Tensor qkv, torch::Tensor pos, torch::Tensor table, torch::Tensor kc, torch::Tensor vc,
                 torch::Tensor len) {
  check_rowmajor(qkv, "qkv");
  check_cache(kc, "k_cache");
  check_cache(vc, "v_cache");
  check_len(len);
  const int64_t B = kc.size(0), Tmax = kc.size(1), H = kc.size(2), hd = kc.size(3);
  TORCH_CHECK(qkv.size(0) == B && qkv.size(1) == 3 * H * hd && qkv.stride(0) % 8 == 0 &&
                  qkv.scalar_type() == torch::kBFloat16 && hd % 16 == 0,
              "rope_append: qkv must be [B, 3*H*hd] bf16, hd % 16 == 0");
  TORCH_CHECK(pos.is_cuda() && pos.scalar_type() == torch::kInt64 && pos.is_contiguous() && pos.numel() == B,
              "rope_append: pos must be contiguous int64 [B]");
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == torch::kFloat32 && table.is_contiguous() &&
                  table.size(1) == hd,
              "rope_append: table must be fp32 [maxlen, hd]");
  const at::DeviceGuard g(qkv.device());
  dpfs_rope_append(qkv.data_ptr(), qkv.stride(0), pos.data_ptr<int64_t>(), table.data_ptr<float>(), kc.data_ptr(),
                   vc.data_ptr(), len.data_ptr<int>(), (int)B, (int)H, (int)hd, (int)Tmax, stream());
}

// Per-tensor fp8 quantisation with current scaling: (q, inv) with q = sat(x * FMAX / amax)
// in float8_e4m3fn (fmt 0) or float8_e5m2 (fmt 1), inv = amax / FMAX as an fp32 0-d tensor
// (the scale torch._scaled_mm multiplies back).  No host synchronisation.
std::vector<torch::Tensor> fp8_quant(torch::Tensor x, int64_t fmt) {
  check_cuda(x, "x");
  TORCH_CHECK(x.scalar_type() == torch::kBFloat16 && x.is_contiguous() && x.numel() % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "fp8_quant: x must be contiguous bf16 with numel % 8 == 0");
  TORCH_CHECK(fmt == 0 || fmt == 1, "fp8_quant: fmt 0 (e4m3) or 1 (e5m2)");
  const at::DeviceGuard g(x.device());
  auto q = torch::empty(x.sizes(), x.options().dtype(fmt == 0 ? at::kFloat8_e4m3fn : at::kFloat8_e5m2));
  auto inv = torch::empty({}, x.options().dtype(torch::kFloat32));
  auto work = torch::empty({dpfs_fp8_work_floats()}, x.options().dtype(torch::kFloat32));
  if (x.numel())
    dpfs_fp8_quant(x.data_ptr(), x.numel(), (int)fmt, q.data_ptr(), inv.data_ptr<float>(), work.data_ptr<float>(),
                   stream());
  else
    inv.fill_(1.0);
  return {q, inv};
}

// *len += 1 and pos[:] = *len on the device (end of a decode step; graph-replayable).
void step_advance(torch::Tensor len, torch::Tensor pos) {
  check_len(len);
  check_cuda(pos, "pos");
  TORCH_CHECK(pos.scalar_type() == torch::kInt64 && pos.is_contiguous(), "pos must be contiguous int64");
  const at::DeviceGuard g(len.device());
  dpfs_step_advance(len.data_ptr<int>(), pos.data_ptr<int64_t>(), (int)pos.numel(), stream());
}

// ------------------------------------------------------------- xGMI collectives (comm/) --
void* xgmi_ptr(int64_t h) {
  TORCH_CHECK(h != 0, "xgmi: null communicator");
  return reinterpret_cast<void*>(h);
}

py::tuple xgmi_create(int64_t rank, int64_t world, int64_t cap_bytes, int64_t nslots) {
  std::string hb((size_t)dpfs_xgmi_handle_bytes(), '\0');
  void* h = dpfs_xgmi_create((int)rank, (int)world, cap_bytes, (int)nslots, &hb[0]);
  TORCH_CHECK(h != nullptr, "xgmi_create failed: ", dpfs_xgmi_last_error());
  return py::make_tuple(reinterpret_cast<int64_t>(h), py::bytes(hb));
}

void xgmi_open(int64_t h, py::bytes all_handles) {
  std::string s = all_handles;
  TORCH_CHECK(s.size() % dpfs_xgmi_handle_bytes() == 0, "xgmi_open: handle blob size");
  TORCH_CHECK(dpfs_xgmi_open(xgmi_ptr(h), s.data()) == 0, "xgmi_open failed: ", dpfs_xgmi_last_error());
}

// op 0 all-reduce (out may be x), 1 reduce-scatter (out = x.numel()/W elements),
// 2 all-gather (out = W * x.numel() elements), 3 one-shot all-reduce (out may be x; up to the
// one-shot capacity, unstaged); launched on the current stream.
// A staging slot as a non-owning uint8 tensor of `cap` bytes on `device` (the communicator
// owns the memory; the Python side keeps the communicator alive as long as the views).
torch::Tensor xgmi_slot_tensor(int64_t h, int64_t slot, int64_t cap, torch::Device device) {
  void* p = dpfs_xgmi_slot(xgmi_ptr(h), (int)slot);
  TORCH_CHECK(p != nullptr, "xgmi: no staging slot ", slot);
  return torch::from_blob(p, {cap}, torch::TensorOptions().dtype(torch::kUInt8).device(device));
}

void xgmi_run(int64_t h, int64_t op, torch::Tensor x, torch::Tensor out, int64_t world, double timeout_s,
              int64_t slot) {
  TORCH_CHECK(op >= 0 && op <= 3, "xgmi_run: op");
  check_cuda(x, "x");
  check_cuda(out, "out");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous(), "xgmi_run: contiguous tensors");
  TORCH_CHECK(x.scalar_type() == out.scalar_type(), "xgmi_run: dtype mismatch");
  const int dt = dcode(x);
  const int64_t vec = dt == 1 ? 8 : 4;
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "xgmi_run: 16-byte aligned buffers");
  const int64_t n = x.numel();
  TORCH_CHECK(n > 0 && n % vec == 0, "xgmi_run: numel must be a positive multiple of ", vec);
  int64_t total, part;
  if (op == 3) {
    TORCH_CHECK(out.numel() == n && slot < 0, "xgmi one-shot all_reduce: out numel, no staging");
    total = n;
    part = n;
  } else if (op == 0) {
    TORCH_CHECK(out.numel() == n, "xgmi all_reduce: out numel");
    total = n;
    part = ((n + world * vec - 1) / (world * vec)) * vec;
  } else if (op == 1) {
    TORCH_CHECK(n % (world * vec) == 0 && out.numel() * world == n, "xgmi reduce_scatter: sizes");
    total = n;
    part = n / world;
  } else {
    TORCH_CHECK(out.numel() == n * world, "xgmi all_gather: out numel");
    total = n * world;
    part = n;
  }
  const at::DeviceGuard g(x.device());
  TORCH_CHECK(dpfs_xgmi_run(xgmi_ptr(h), (int)op, dt, x.data_ptr(), out.data_ptr(), total, part, timeout_s,
                            (int)slot, stream()) == 0,
              "xgmi_run failed: ", dpfs_xgmi_last_error());
}

// ------------------------------------------------------- native RCCL communicator (comm/) --
void* rccl_ptr(int64_t h) {
  TORCH_CHECK(h != 0, "rccl: null communicator");
  return reinterpret_cast<void*>(h);
}

int rccl_dtype(const torch::Tensor& t) {   // ncclDataType_t values (rccl.h)
  switch (t.scalar_type()) {
    case torch::kBFloat16: return 9;
    case torch::kFloat32: return 7;
    case torch::kFloat16: return 6;
    case torch::kFloat64: return 8;
    case torch::kInt64: return 4;
    case torch::kInt32: return 2;
    case torch::kUInt8: return 1;
    default: TORCH_CHECK(false, "rccl: unsupported dtype ", t.scalar_type());
  }
  return -1;
}

void rccl_check(int rc, const char* what) { TORCH_CHECK(rc == 0, what, " failed: ", dpfs_rccl_last_error()); }

py::bytes rccl_unique_id() {
  std::string b((size_t)dpfs_rccl_id_bytes(), '\0');
  rccl_check(dpfs_rccl_unique_id(&b[0]), "ncclGetUniqueId");
  return py::bytes(b);
}

int64_t rccl_init(py::bytes id, int64_t nranks, int64_t rank) {
  std::string b = id;
  TORCH_CHECK((int)b.size() == dpfs_rccl_id_bytes(), "rccl_init: unique id size");
  void* c = nullptr;
  {
    py::gil_scoped_release nogil;   // blocks until every rank has joined
    rccl_check(dpfs_rccl_init(b.data(), (int)nranks, (int)rank, &c), "ncclCommInitRank");
  }
  return reinterpret_cast<int64_t>(c);
}

// Collectives on the CURRENT HIP stream (the Python side selects its side stream).
void rccl_all_reduce(int64_t h, torch::Tensor x, torch::Tensor out, int64_t op) {
  check_cuda(x, "x");
  check_cuda(out, "out");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && x.numel() == out.numel() &&
                  x.scalar_type() == out.scalar_type(), "rccl all_reduce: contiguous, same size and dtype");
  const at::DeviceGuard g(x.device());
  rccl_check(dpfs_rccl_all_reduce(rccl_ptr(h), x.data_ptr(), out.data_ptr(), (size_t)x.numel(), rccl_dtype(x),
                                  (int)op, stream()), "ncclAllReduce");
}

void rccl_reduce_scatter(int64_t h, torch::Tensor out, torch::Tensor x, int64_t world, int64_t op) {
  check_cuda(x, "x");
  check_cuda(out, "out");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && out.numel() * world == x.numel() &&
                  x.scalar_type() == out.scalar_type(), "rccl reduce_scatter: out = in / world elements");
  const at::DeviceGuard g(x.device());
  rccl_check(dpfs_rccl_reduce_scatter(rccl_ptr(h), x.data_ptr(), out.data_ptr(), (size_t)out.numel(), rccl_dtype(x),
                                      (int)op, stream()), "ncclReduceScatter");
}

void rccl_all_gather(int64_t h, torch::Tensor out, torch::Tensor x, int64_t world) {
  check_cuda(x, "x");
  check_cuda(out, "out");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && x.numel() * world == out.numel() &&
                  x.scalar_type() == out.scalar_type(), "rccl all_gather: out = world x in elements");
  const at::DeviceGuard g(x.device());
  rccl_check(dpfs_rccl_all_gather(rccl_ptr(h), x.data_ptr(), out.data_ptr(), (size_t)x.numel(), rccl_dtype(x),
                                  stream()), "ncclAllGather");
}

void rccl_broadcast(int64_t h, torch::Tensor t, int64_t root) {
  check_cuda(t, "t");
  TORCH_CHECK(t.is_contiguous(), "rccl broadcast: contiguous tensor");
  const at::DeviceGuard g(t.device());
  rccl_check(dpfs_rccl_broadcast(rccl_ptr(h), t.data_ptr(), t.data_ptr(), (size_t)t.numel(), rccl_dtype(t),
                                 (int)root, stream()), "ncclBroadcast");
}

// ---- hipBLASLt, driven directly (blas/blaslt.hip) ----
// layout 0 NT: out[M,N] bf16 = a[M,K] b[N,K]^T (+ bias fp32[N]);  1 NN: out = a[M,K] b[K,N];
// 2 TN: out[M,N] fp32 (+)= a[K,M]^T b[K,N].  Operands contiguous bf16.
int64_t lt_algos(int64_t layout, int64_t M, int64_t N, int64_t K, bool bias) {
  return dpfs_lt_algos((int)layout, M, N, K, bias ? 1 : 0);
}

void lt_run(int64_t layout, torch::Tensor a, torch::Tensor b, torch::Tensor out, c10::optional<torch::Tensor> bias,
            int64_t algo, bool accumulate) {
  TORCH_CHECK(layout >= 0 && layout <= 2, "lt_run: layout 0 (NT), 1 (NN) or 2 (TN)");
  for (const torch::Tensor* t : {&a, &b, &out}) {
    check_cuda(*t, "lt_run operand");
    TORCH_CHECK(t->dim() == 2 && t->is_contiguous(), "lt_run: 2-D contiguous operands");
  }
  TORCH_CHECK(a.scalar_type() == torch::kBFloat16 && b.scalar_type() == torch::kBFloat16, "lt_run: bf16 operands");
  int64_t M, N, K;
  if (layout == 0) {
    M = a.size(0), K = a.size(1), N = b.size(0);
    TORCH_CHECK(b.size(1) == K, "lt_run NT: a [M,K], b [N,K]");
  } else if (layout == 1) {
    M = a.size(0), K = a.size(1), N = b.size(1);
    TORCH_CHECK(b.size(0) == K, "lt_run NN: a [M,K], b [K,N]");
  } else {
    K = a.size(0), M = a.size(1), N = b.size(1);
    TORCH_CHECK(b.size(0) == K, "lt_run TN: a [K,M], b [K,N]");
  }
  TORCH_CHECK(out.size(0) == M && out.size(1) == N, "lt_run: out must be [M, N]");
  TORCH_CHECK(out.scalar_type() == (layout == 2 ? torch::kFloat32 : torch::kBFloat16),
              "lt_run: out fp32 for TN, bf16 otherwise");
  TORCH_CHECK(!accumulate || layout == 2, "lt_run: accumulate is TN only");
  const float* bp = nullptr;
  if (bias.has_value()) {
    TORCH_CHECK(layout == 0, "lt_run: bias is NT only");
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->is_contiguous() && bias->numel() == N,
                "lt_run: bias fp32 [N] contiguous");
    bp = bias->data_ptr<float>();
  }
  TORCH_CHECK(a.device() == b.device() && a.device() == out.device(), "lt_run: operands on one device");
  const at::DeviceGuard g(a.device());
  const int n = dpfs_lt_algos((int)layout, M, N, K, bp ? 1 : 0);
  TORCH_CHECK(algo >= 0 && algo < n, "lt_run: algorithm ", algo, " of ", n, " (", dpfs_lt_last_error(), ")");
  const long long wsb = dpfs_lt_workspace((int)layout, M, N, K, bp ? 1 : 0, (int)algo);
  torch::Tensor ws;
  if (wsb > 0) ws = torch::empty({wsb}, a.options().dtype(torch::kUInt8));
  const int st = dpfs_lt_run((int)layout, M, N, K, bp, (int)algo, a.data_ptr(), b.data_ptr(), out.data_ptr(),
                             accumulate ? 1.f : 0.f, wsb > 0 ? ws.data_ptr() : nullptr, wsb > 0 ? wsb : 0, stream());
  TORCH_CHECK(st == 0, "hipBLASLt: ", dpfs_lt_last_error());
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 (MI355X) HIP kernels of distributed_pytorch_from_scratch_amd";
  m.def("gemm_nt", &gemm_nt, py::arg("a"), py::arg("b"), py::arg("bias") = py::none(),
        py::arg("rope_pos") = py::none(), py::arg("rope_tab") = py::none(), py::arg("rope_heads") = 0,
        py::arg("rope_hd") = 0, py::arg("out") = py::none(), py::arg("variant") = 0);
  m.def("gemm_nn", &gemm_nn, py::arg("a"), py::arg("b"), py::arg("out") = py::none(), py::arg("variant") = 0);
  m.def("gemm_force", [](int cfg, int splits) { dpfs_gemm_force(cfg, splits); },
        "force the v2 tile config (-1 auto, 0 = 256x256, 1 = 256x128) and K-splits (0 auto)");
  m.def("gemm4_ablate", [](int v) { dpfs_gemm4_ablate(v); }, "timing-only: 1 = drop stores, 2 = zero operands");
  m.def("attn_diag", [](torch::Tensor t) { dpfs_attn_diag(t.defined() && t.numel() ? t.data_ptr() : nullptr); },
        "int64 buffer of the DIAG builds (attn_fwd / attn_bwd impl 5): per-wave s_memtime splits");
  m.def("gemm4_diag", [](torch::Tensor t) { dpfs_gemm4_diag(t.defined() && t.numel() ? t.data_ptr() : nullptr); },
        "int64 buffer [grid*4*4] for the DIAG build's per-wave cycle split (gemm4_ablate bit 16)");
  m.def("gemm_tn_group", &gemm_tn_group, py::arg("a"), py::arg("b"), py::arg("outs"), py::arg("acc"),
        py::arg("a2") = py::none(), py::arg("b2") = py::none());
  m.def("gemm_tn_splits", [](int M, int N, int K) { return dpfs_gemm_tn_splits(M, N, K); },
        "K-split count of the TN (weight-gradient) plan for an M x N output over K");
  m.def("attn_prefetch", [](int v) { dpfs_attn_prefetch(v); },
        "head_dim-64 attention backward, next block's operands fetched ahead: bit 0 = dK/dV, bit 1 = dQ (3 default; A/B)");
  m.def("gemm4_swb_depth", [](int v) { dpfs_gemm4_swb_depth(v); },
        "SwiGLU-backward epilogue of the down-projection dgrad: gate / up row blocks in flight (2 default, 1 = A/B)");
  m.def("gemm_sk_error", [](bool reset) { return dpfs_gemm4_sk_error(reset ? 1 : 0); }, py::arg("reset") = false,
        "sticky host-mapped word: 1 when a stream-K consumer's bounded wait for its producer's partial timed out "
        "(that GEMM's output is wrong); read without a device sync");
  m.def("gemm_sk_starve", [](bool on) { dpfs_gemm4_sk_starve(on ? 1 : 0); },
        "test hook: the next stream-K launch's producers never raise their flags, so every consumer wait times out");
  m.def("gemm_sk_applies", [](int64_t M, int64_t N, int64_t K) { return dpfs_gemm4_sk_ws((int)M, (int)N, (int)K) > 0; },
        "whether the stream-K bf16 kernel (variant 8 / 12) applies to an M x N x K NT / NN GEMM on this device");
  m.def("gemm4_m32k", [](int v) { dpfs_gemm4_m32k(v); },
        "NN / NT 256-wide main loop of the v4 GEMM: bit 0 = 32x32x16 MFMAs for the fp32 (split-K) output, bit 1 = for "
        "the bf16 (+ bias) output, 0 = 16x16x32 (default; measured faster in the step)");
  m.def("gemm4_m32", [](int v) { dpfs_gemm4_m32(v); },
        "TN main loop of the v4 GEMM: 1 = 32x32x16 MFMAs (default), 0 = 16x16x32 (A/B probes)");
  m.def("gemm4_br", [](int v) { dpfs_gemm4_br(v); },
        "rows of MFMAs before each step's barrier in the plain v4 kernels (0, 1, 2 = default; A/B runs)");
  m.def("gemm4_sched", [](int v) { dpfs_gemm4_sched(v); },
        "v4 main-loop variant: 0 = default (descriptor-advancing DMA where K ranges allow, one piece per MFMA "
        "row), 1 = two pieces per row in rows 4-7, 2 = per-lane K checks everywhere (the pre-FAST stream)");
  m.def("gemm4_br_tn", [](int v) { dpfs_gemm4_br_tn(v); },
        "blocks of 4 MFMAs before each step's barrier in the 32x32x16 (TN weight-gradient) main loop (0 default, 1, 2; A/B)");
  m.def("gemm4_group_m", [](int v) { dpfs_gemm4_group_m(v); }, "v4 tile-row group size of the item order (default 4)");
  m.def("gemm_v2_sched", [](int v) { dpfs_gemm_v2_sched(v); }, "v2 256x256 schedule (-1 per-layout default, 0..4 see gemm2_k SCHED)");
  m.def("gemm_set_impl", [](int v) { dpfs_gemm_set_impl(v); }, "1 = v1 (128x128 register-staged), 2 = v2 (LDS-DMA, one tile per workgroup), 3 = v3 (persistent v2, default)");
  m.def("gemm_tn2", &gemm_tn2, "fp32 c (+)= a0^T b0 + a1^T b1 (reduction dim over two buffers), one split-K launch; None if the plan does not fit",
        py::arg("a0"), py::arg("b0"), py::arg("a1"), py::arg("b1"), py::arg("out") = py::none(),
        py::arg("accumulate") = false, py::arg("variant") = 0);
  m.def("gemm_tn", &gemm_tn, py::arg("a"), py::arg("b"), py::arg("out") = py::none(), py::arg("accumulate") = false,
        py::arg("variant") = 0);
  m.def("bias_grad", &bias_grad);
  m.def("add_bias_", &add_bias_);
  m.def("bias_residual", &bias_residual);
  m.def("rmsnorm_fwd", &rmsnorm_fwd);
  m.def("add_rmsnorm_fwd", &add_rmsnorm_fwd, py::arg("y"), py::arg("bias"), py::arg("res"), py::arg("w"),
        py::arg("eps"));
  m.def("rmsnorm_bwd", &rmsnorm_bwd, py::arg("dy"), py::arg("x"), py::arg("w"), py::arg("rstd"),
        py::arg("dres") = py::none(), py::arg("dbias") = py::none(), py::arg("dw_out") = py::none());
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("layernorm_bwd", &layernorm_bwd);
  m.def("swiglu_fwd", &swiglu_fwd, py::arg("gu"), py::arg("perm") = false);
  m.def("swiglu_bwd", &swiglu_bwd, py::arg("dh"), py::arg("gu"), py::arg("dbias") = py::none(),
        py::arg("perm") = false);
  m.def("gemm_nn_swiglu_bwd", &gemm_nn_swiglu_bwd, py::arg("dy"), py::arg("w"), py::arg("gu"),
        py::arg("dbias") = py::none(), py::arg("perm") = true);
  m.def("gemm_nt_swiglu", &gemm_nt_swiglu,
        "gate|up NT GEMM (rows interleaved in 64-row blocks) with SwiGLU in the epilogue: [gu, h] or []",
        py::arg("a"), py::arg("b"), py::arg("bias") = py::none());
  m.def("rope_", &rope_, py::arg("qkv"), py::arg("positions"), py::arg("table"), py::arg("n_rot_heads"),
        py::arg("head_dim"), py::arg("inverse") = false);
  m.def("attn_fwd", &attn_fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("scale"), py::arg("causal") = true,
        py::arg("impl") = 0,
        "flash attention forward; impl (per call): 0 = auto (32x32x16 LDS-DMA ring at hd 64 / 128, "
        "16x16x32 register-staged at hd 32), 1 = 16x16x32 register-staged, 4 = 32x32x16 ring, 5 = its DIAG build");
  m.def("attn_bwd", &attn_bwd, py::arg("dout"), py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"),
        py::arg("lse"), py::arg("scale"), py::arg("causal"), py::arg("dq"), py::arg("dk"), py::arg("dv"),
        py::arg("rope_pos") = py::none(), py::arg("rope_tab") = py::none(), py::arg("dbias") = py::none(),
        py::arg("impl") = 0,
        "flash attention backward; impl (per call): 0 = auto (dq3 + dkdv3 at hd 64 / 128, dq + dkdv2 at hd 32), "
        "2 = dq + dkdv2 (16x16x32), 4 = dq3 + dkdv3 (32x32x16), 5 = 4 with the dK/dV DIAG build, 6 = the fused "
        "head_dim-64 backward (delta pass, one dK/dV/dQ kernel, dQ partial reduction)");
  m.def("ce_finalize", &ce_finalize, py::arg("stats"), py::arg("targets"), py::arg("ignore_index"), py::arg("acc"),
        py::arg("loss"), py::arg("first"), py::arg("last"),
        "CE loss bookkeeping from gathered (nsh, M, 3) statistics: returns (lse, valid); running sums in acc");
  m.def("ce_valid_scale", &ce_valid_scale, py::arg("targets"), py::arg("ignore_index"),
        "(gs, n_valid): per-row 1 / max(#valid, 1) on valid rows (0 on ignored), and max(#valid, 1)");
  m.def("emb_sort", &emb_sort, py::arg("ids"), py::arg("vocab_start"), py::arg("v_local"),
        "(perm, seg): the ids' stable order by local vocab row (out-of-shard ids last) and each row's segment "
        "start, int64 (deterministic radix sort on HIP kernels)");
  m.def("gemm_f32", &gemm_f32, py::arg("a"), py::arg("b"), py::arg("layout"), py::arg("bias") = py::none(),
        py::arg("out") = py::none(), py::arg("accumulate") = false,
        "fp32-input MFMA GEMM (v_mfma_f32_32x32x2_f32, exact products): layout 0 = a b^T (+ bias), 1 = a b, 2 = a^T b "
        "(+=); fp32 or bf16 operands of any alignment (bf16: the shapes the bf16 MFMA kernels decline)");
  m.def("attn_fwd_f32", &attn_fwd_f32, "fp32 causal flash attention forward: (o, lse)");
  m.def("attn_bwd_f32", &attn_bwd_f32, py::arg("dout"), py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"),
        py::arg("lse"), py::arg("scale"), py::arg("causal"), py::arg("dq"), py::arg("dk"), py::arg("dv"),
        py::arg("rope_pos") = py::none(), py::arg("rope_tab") = py::none(), py::arg("dbias") = py::none(),
        "fp32 flash attention backward (dQ kernel, then dK/dV), optional inverse RoPE and QKV bias gradient");
  m.def("occupy", [](int64_t blocks, double us) { dpfs_occupy((int)blocks, us, stream()); }, py::arg("blocks"),
        py::arg("us"),
        "collective stand-in on the current stream: `blocks` resident 1024-thread workgroups for `us` microseconds");
  m.def("ce_grad_scale", &ce_grad_scale, py::arg("valid"), py::arg("gloss"), py::arg("n_valid"),
        "gs = valid * gloss / n_valid (the CE backward's per-row loss gradient; device scalars, one launch)");
  m.def("attn_stagger", [](int v) { dpfs_attn_stagger(v); },
        "A/B hook: odd workgroups of the v3 attention backward kernels start v x 8k cycles late (0 default)");
  m.def("embedding_fwd", &embedding_fwd);
  m.def("embedding_bwd_sorted", &embedding_bwd_sorted, py::arg("dout"), py::arg("ids"), py::arg("v_local"),
        py::arg("vocab_start"), py::arg("out") = py::none(), py::arg("accumulate") = false,
        py::arg("perm") = py::none(), py::arg("seg") = py::none(),
        "deterministic embedding gradient (sorted ids, one wave per vocab row; writes or adds every row)");
  m.def("embedding_bwd", &embedding_bwd, py::arg("dout"), py::arg("ids"), py::arg("v_local"), py::arg("vocab_start"),
        py::arg("out") = py::none());
  m.def("ce_fwd_stats", &ce_fwd_stats);
  m.def("ce_fused", &ce_fused, py::arg("logits"), py::arg("targets"), py::arg("gscale"), py::arg("vocab_start"),
        py::arg("vocab_valid"), py::arg("dbias") = py::none());
  m.def("ce_bwd", &ce_bwd, py::arg("logits"), py::arg("targets"), py::arg("lse"), py::arg("gscale"),
        py::arg("vocab_start"), py::arg("vocab_valid"), py::arg("out"), py::arg("dbias") = py::none());
  m.def("adam_build", &adam_build);
  m.def("adam_step", &adam_step, py::arg("desc"), py::arg("chunks"), py::arg("lr"), py::arg("beta1"),
        py::arg("beta2"), py::arg("eps"), py::arg("weight_decay"), py::arg("step"), py::arg("grad_scale") = 1.0,
        py::arg("dscale") = py::none());
  m.def("grad_sumsq", &grad_sumsq);
  m.def("adam_patch_grads", &adam_patch_grads, py::arg("desc"), py::arg("grads"));
  m.def("attn_decode", &attn_decode, py::arg("q"), py::arg("k_cache"), py::arg("v_cache"), py::arg("len"),
        py::arg("scale"));
  m.def("kv_append", &kv_append, py::arg("qkv"), py::arg("k_cache"), py::arg("v_cache"), py::arg("len"));
  m.def("step_advance", &step_advance, py::arg("len"), py::arg("pos"));
  m.def("lt_algos", &lt_algos, py::arg("layout"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("bias") = false,
        "hipBLASLt heuristic algorithms for a problem (0 NT, 1 NN, 2 TN)");
  m.def("lt_run", &lt_run, py::arg("layout"), py::arg("a"), py::arg("b"), py::arg("out"), py::arg("bias") = py::none(),
        py::arg("algo") = 0, py::arg("accumulate") = false);
  m.def("fp8_quant", &fp8_quant, py::arg("x"), py::arg("fmt") = 0);
  m.def("gemv_nt_ok", &gemv_nt_ok, py::arg("x"), py::arg("w"), py::arg("swiglu") = false);
  m.def("gemv_nt", &gemv_nt, py::arg("x"), py::arg("w"), py::arg("bias") = py::none(), py::arg("swiglu") = false);
  m.def("rope_append", &rope_append, py::arg("qkv"), py::arg("pos"), py::arg("table"), py::arg("k_cache"),
        py::arg("v_cache"), py::arg("len"));
  m.def("xgmi_create", &xgmi_create, "allocate IPC buffers: -> (handle, ipc handle bytes)");
  m.def("xgmi_open", &xgmi_open, "map every peer's buffers (rank-ordered concatenated handle bytes)");
  m.def("xgmi_run", &xgmi_run, py::arg("h"), py::arg("op"), py::arg("x"), py::arg("out"), py::arg("world"),
        py::arg("timeout_s") = 120.0, py::arg("slot") = -1);
  m.def("xgmi_one_shot_capacity", [](int64_t h) { return dpfs_xgmi_one_shot_capacity(xgmi_ptr(h)); });
  m.def("xgmi_slot_tensor", &xgmi_slot_tensor, py::arg("h"), py::arg("slot"), py::arg("cap"), py::arg("device"));
  m.def("xgmi_set_blocks", [](int64_t h, int b) { dpfs_xgmi_set_blocks(xgmi_ptr(h), b); });
  m.def("xgmi_capacity", [](int64_t h) { return dpfs_xgmi_capacity(xgmi_ptr(h)); });
  m.def("xgmi_error", [](int64_t h) { return dpfs_xgmi_error(xgmi_ptr(h)); });
  m.def("xgmi_clear_error", [](int64_t h) { dpfs_xgmi_clear_error(xgmi_ptr(h)); });
  m.def("xgmi_destroy", [](int64_t h) { dpfs_xgmi_destroy(xgmi_ptr(h)); });
  m.def("rccl_unique_id", &rccl_unique_id, "ncclGetUniqueId -> bytes");
  m.def("rccl_init", &rccl_init, py::arg("id"), py::arg("nranks"), py::arg("rank"),
        "ncclCommInitRank on the current device -> communicator handle");
  m.def("rccl_all_reduce", &rccl_all_reduce, py::arg("h"), py::arg("x"), py::arg("out"), py::arg("op") = 0);
  m.def("rccl_reduce_scatter", &rccl_reduce_scatter, py::arg("h"), py::arg("out"), py::arg("x"), py::arg("world"),
        py::arg("op") = 0);
  m.def("rccl_all_gather", &rccl_all_gather, py::arg("h"), py::arg("out"), py::arg("x"), py::arg("world"));
  m.def("rccl_broadcast", &rccl_broadcast, py::arg("h"), py::arg("t"), py::arg("root"));
  m.def("rccl_group_start", []() { TORCH_CHECK(dpfs_rccl_group_start() == 0, "ncclGroupStart"); });
  m.def("rccl_group_end", []() { rccl_check(dpfs_rccl_group_end(), "ncclGroupEnd"); });
  m.def("rccl_async_error", [](int64_t h) {
    return dpfs_rccl_async_error(rccl_ptr(h)) == 0 ? std::string() : std::string(dpfs_rccl_last_error());
  });
  m.def("rccl_destroy", [](int64_t h) { rccl_check(dpfs_rccl_destroy(rccl_ptr(h)), "ncclCommDestroy"); });
}
