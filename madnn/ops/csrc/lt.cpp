// Epilogue-fused Linear on hipBLASLt (host code; the GEMM itself is a library kernel).
//
// GPT-2's MLP spends two standalone elementwise passes around its GEMMs: the tanh-GELU
// after c_fc and the residual add after c_proj (profiles/r1_gpt2m_dp1_k11.md).  hipBLASLt
// fuses both into the GEMM's epilogue:
//
//   y   = gelu(x W^T + b)          (HIPBLASLT_EPILOGUE_GELU_AUX_BIAS)
//   pre = x W^T + b                 (the AUX output, what the K11 GELU backward reads)
//   y   = x W^T + b + residual      (beta = 1 with C = residual, D a fresh buffer)
//
// Row-major Y[M,N] = X[M,K] W[N,K]^T is the column-major product D[N,M] = op(A) B with
// A = W (stored K x N, transposed), B = X (K x M), so the bias (length N = rows of D) is the
// epilogue's broadcast vector.  The handle and workspace are PyTorch's own (same hipBLASLt
// instance, per-stream workspace); matmul descriptors and the heuristic's algorithm are cached
// per (M, N, K, epilogue, dtypes).
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

namespace at {
namespace cuda {
hipblasLtHandle_t getCurrentCUDABlasLtHandle();
void* getCUDABlasLtWorkspace();
size_t getCUDABlasLtWorkspaceSize();
}  // namespace cuda
}  // namespace at

namespace {

#define LT_CHECK(expr)                                                                         \
  do {                                                                                         \
    hipblasStatus_t _st = (expr);                                                              \
    TORCH_CHECK(_st == HIPBLAS_STATUS_SUCCESS, "hipBLASLt call failed (", (int)_st, "): " #expr); \
  } while (0)

hipDataType lt_type(at::ScalarType t) {
  switch (t) {
    case at::kBFloat16: return HIP_R_16BF;
    case at::kHalf: return HIP_R_16F;
    case at::kFloat: return HIP_R_32F;
    default: TORCH_CHECK(false, "lt_linear: unsupported dtype ", t);
  }
  return HIP_R_32F;
}

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo;
  size_t ws = 0;
  int n = 0;  // candidates the heuristic returned
};

using Key = std::tuple<int64_t, int64_t, int64_t, int, int, int, int, int, size_t, int>;  // [7]: w given [K, N], [9]: algo
constexpr int kMaxAlgos = 16;
std::map<Key, Plan> g_plans;
std::mutex g_mu;

Plan& get_plan(hipblasLtHandle_t h, int64_t M, int64_t N, int64_t K, hipblasLtEpilogue_t epi, hipDataType dt,
               hipDataType bias_dt, bool has_c, size_t ws_cap, const void* bias_ptr, void* aux_ptr,
               bool w_kn = false, int algo = 0, int* n_algos = nullptr) {
  Key key{M, N, K, (int)epi, (int)dt, (int)bias_dt, (int)has_c, w_kn ? 1 : 0, ws_cap, algo};
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_plans.find(key);
  if (it != g_plans.end()) {
    if (n_algos != nullptr) *n_algos = it->second.n;
    return it->second;
  }
  Plan p;
  LT_CHECK(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t ta = w_kn ? HIPBLAS_OP_N : HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)));
  if (epi != HIPBLASLT_EPILOGUE_DEFAULT && epi != HIPBLASLT_EPILOGUE_GELU && epi != HIPBLASLT_EPILOGUE_GELU_AUX) {
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bias_dt, sizeof(bias_dt)));
  }
  if (bias_ptr != nullptr) {  // set before the heuristic: solution selection looks at it
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias_ptr, sizeof(bias_ptr)));
  }
  if (epi == HIPBLASLT_EPILOGUE_GELU_AUX_BIAS || epi == HIPBLASLT_EPILOGUE_GELU_AUX) {
    int64_t ld = N;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld)));
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &dt, sizeof(dt)));
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux_ptr,
                                             sizeof(aux_ptr)));
  }
  if (w_kn) {
    LT_CHECK(hipblasLtMatrixLayoutCreate(&p.a, dt, N, K, N));  // W [K, N] row-major: N x K col-major, op N
  } else {
    LT_CHECK(hipblasLtMatrixLayoutCreate(&p.a, dt, K, N, K));  // W [N, K] row-major: K x N col-major, op T
  }
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.b, dt, K, M, K));  // X: K x M col-major
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.c, dt, N, M, N));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&p.d, dt, N, M, N));
  hipblasLtMatmulPreference_t pref;
  LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t cap = ws_cap;
  LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &cap, sizeof(cap)));
  // the heuristic's ranked candidates: `algo` picks one (0 = its first choice; a per-shape timed index
  // from the tuning table can name a faster one, madnn.ops.lt_algo)
  hipblasLtMatmulHeuristicResult_t res[kMaxAlgos];
  int n = 0;
  LT_CHECK(hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.a, p.b, p.c, p.d, pref, algo > 0 ? kMaxAlgos : 1, res, &n));
  hipblasLtMatmulPreferenceDestroy(pref);
  TORCH_CHECK(n > 0, "lt_linear: hipBLASLt has no algorithm for M=", M, " N=", N, " K=", K, " epilogue=", (int)epi);
  if (n_algos != nullptr) {  // lt_algo_count's query: the count, and the last candidate as the plan
    *n_algos = n;
    algo = algo < n ? algo : n - 1;
  }
  TORCH_CHECK(algo < n, "lt_linear: algorithm index ", algo, " of ", n);
  p.n = n;
  p.algo = res[algo].algo;
  p.ws = res[algo].workspaceSize;
  (void)has_c;
  return g_plans.emplace(key, p).first->second;
}

// x [M, K], w [N, K] (both contiguous, same dtype), bias [N] or None, residual [M, N] or None.
// w_kn: w is given as [K, N] instead (y = x @ w, e.g. a Linear's data gradient dy @ W, no transposed copy).
// Returns (y [M, N], pre [M, N] when gelu && want_pre, else an empty tensor).
std::tuple<at::Tensor, at::Tensor> lt_linear(const at::Tensor& x, const at::Tensor& w,
                                             const c10::optional<at::Tensor>& bias,
                                             const c10::optional<at::Tensor>& residual, bool gelu, bool want_pre,
                                             bool w_kn, int64_t algo) {
  TORCH_CHECK(algo >= 0 && algo < kMaxAlgos, "lt_linear: algo in [0, ", kMaxAlgos, ")");
  TORCH_CHECK(x.is_cuda() && w.is_cuda() && x.dim() == 2 && w.dim() == 2, "lt_linear: 2-D HIP tensors");
  TORCH_CHECK(x.is_contiguous() && w.is_contiguous(), "lt_linear: contiguous x and w");
  TORCH_CHECK(x.scalar_type() == w.scalar_type(), "lt_linear: x and w dtypes differ");
  const int64_t M = x.size(0), K = x.size(1), N = w_kn ? w.size(1) : w.size(0);
  TORCH_CHECK((w_kn ? w.size(0) : w.size(1)) == K, "lt_linear: shape mismatch");
  const bool has_bias = bias.has_value() && bias->defined();
  const bool has_res = residual.has_value() && residual->defined();
  if (has_bias) TORCH_CHECK(bias->is_contiguous() && bias->numel() == N, "lt_linear: bias [N]");
  if (has_res)
    TORCH_CHECK(residual->is_contiguous() && residual->size(0) == M && residual->size(1) == N &&
                    residual->scalar_type() == x.scalar_type(), "lt_linear: residual [M, N] of x's dtype");
  hipblasLtEpilogue_t epi = HIPBLASLT_EPILOGUE_DEFAULT;
  if (gelu) {
    epi = want_pre ? (has_bias ? HIPBLASLT_EPILOGUE_GELU_AUX_BIAS : HIPBLASLT_EPILOGUE_GELU_AUX)
                   : (has_bias ? HIPBLASLT_EPILOGUE_GELU_BIAS : HIPBLASLT_EPILOGUE_GELU);
  } else if (has_bias) {
    epi = HIPBLASLT_EPILOGUE_BIAS;
  }
  const hipDataType dt = lt_type(x.scalar_type());
  const hipDataType bdt = has_bias ? lt_type(bias->scalar_type()) : dt;
  const at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  hipblasLtHandle_t h = at::cuda::getCurrentCUDABlasLtHandle();
  const size_t ws_cap = at::cuda::getCUDABlasLtWorkspaceSize();
  void* ws = at::cuda::getCUDABlasLtWorkspace();
  at::Tensor y = at::empty({M, N}, x.options());
  at::Tensor pre;
  if (gelu && want_pre) pre = at::empty({M, N}, x.options());
  Plan& p = get_plan(h, M, N, K, epi, dt, bdt, has_res, ws_cap, has_bias ? bias->data_ptr() : nullptr,
                     pre.defined() ? pre.data_ptr() : nullptr, w_kn, (int)algo);
  if (has_bias) {
    const void* bp = bias->data_ptr();
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp)));
  }
  if (gelu && want_pre) {
    void* ap = pre.data_ptr();
    LT_CHECK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &ap, sizeof(ap)));
  }
  const float alpha = 1.0f, beta = has_res ? 1.0f : 0.0f;
  const void* cptr = has_res ? residual->data_ptr() : y.data_ptr();
  hipStream_t stream = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  LT_CHECK(hipblasLtMatmul(h, p.desc, &alpha, w.data_ptr(), p.a, x.data_ptr(), p.b, &beta, cptr, p.c, y.data_ptr(),
                           p.d, &p.algo, ws, p.ws, stream));
  return {y, pre.defined() ? pre : at::empty({0}, x.options())};
}

// How many ranked candidates the heuristic offers for lt_linear's problem (bias / no bias, no GELU, no
// residual) -- the range of lt_linear's `algo`
int64_t lt_algo_count(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias, bool w_kn) {
  const int64_t M = x.size(0), K = x.size(1), N = w_kn ? w.size(1) : w.size(0);
  const bool has_bias = bias.has_value() && bias->defined();
  const hipDataType dt = lt_type(x.scalar_type());
  const hipDataType bdt = has_bias ? lt_type(bias->scalar_type()) : dt;
  const at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  hipblasLtHandle_t h = at::cuda::getCurrentCUDABlasLtHandle();
  int n = 0;
  get_plan(h, M, N, K, has_bias ? HIPBLASLT_EPILOGUE_BIAS : HIPBLASLT_EPILOGUE_DEFAULT, dt, bdt, false,
           at::cuda::getCUDABlasLtWorkspaceSize(), has_bias ? bias->data_ptr() : nullptr, nullptr, w_kn, kMaxAlgos - 1, &n);
  return n;
}

// How many algorithms hipBLASLt's heuristic offers for an epilogue / type combination
// (0 = unsupported); dtype codes: 0 bf16, 1 fp16, 2 fp32, -1 = leave the attribute unset.
int64_t lt_probe(int64_t M, int64_t N, int64_t K, int64_t epi, int64_t bias_code, int64_t aux_code, bool has_c,
                 int64_t dummy_ptr) {
  auto code = [](int64_t c) { return c == 0 ? HIP_R_16BF : (c == 1 ? HIP_R_16F : HIP_R_32F); };
  hipblasLtHandle_t h = at::cuda::getCurrentCUDABlasLtHandle();
  hipblasLtMatmulDesc_t desc;
  hipblasLtMatrixLayout_t a, b, c, d;
  const hipDataType dt = HIP_R_16BF;
  LT_CHECK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  hipblasLtEpilogue_t e = (hipblasLtEpilogue_t)epi;
  LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e)));
  void* dp = reinterpret_cast<void*>(dummy_ptr);
  if (bias_code >= 0) {
    hipDataType bdt = code(bias_code);
    LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bdt, sizeof(bdt)));
    if (dp) LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &dp, sizeof(dp)));
  }
  if (aux_code >= 0) {
    hipDataType adt = code(aux_code);
    int64_t ld = N;
    LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld)));
    LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, &adt, sizeof(adt)));
    if (dp) LT_CHECK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &dp, sizeof(dp)));
  }
  LT_CHECK(hipblasLtMatrixLayoutCreate(&a, dt, K, N, K));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&b, dt, K, M, K));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&c, dt, N, M, N));
  LT_CHECK(hipblasLtMatrixLayoutCreate(&d, dt, N, M, N));
  hipblasLtMatmulPreference_t pref;
  LT_CHECK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t cap = at::cuda::getCUDABlasLtWorkspaceSize();
  LT_CHECK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &cap, sizeof(cap)));
  hipblasLtMatmulHeuristicResult_t res[8];
  int n = 0;
  hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, desc, a, b, c, d, pref, 8, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  hipblasLtMatrixLayoutDestroy(a);
  hipblasLtMatrixLayoutDestroy(b);
  hipblasLtMatrixLayoutDestroy(c);
  hipblasLtMatrixLayoutDestroy(d);
  hipblasLtMatmulDescDestroy(desc);
  (void)has_c;
  return st == HIPBLAS_STATUS_SUCCESS ? n : -(int64_t)st;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(madnn, m) {
  m.def("lt_linear(Tensor x, Tensor w, Tensor? bias, Tensor? residual, bool gelu, bool want_pre, bool w_kn=False, int algo=0) -> (Tensor, Tensor)");
  m.def("lt_algo_count(Tensor x, Tensor w, Tensor? bias, bool w_kn=False) -> int");
  // no tensor arguments -> nothing to dispatch on: a catch-all kernel
  m.def("lt_probe(int M, int N, int K, int epi, int bias_code, int aux_code, bool has_c, int dummy_ptr) -> int",
        TORCH_FN(lt_probe));
}

TORCH_LIBRARY_IMPL(madnn, CUDA, m) {
  m.impl("lt_linear", lt_linear);
  m.impl("lt_algo_count", lt_algo_count);
}
