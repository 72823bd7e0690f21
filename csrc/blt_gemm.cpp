// Library GEMMs through hipBLASLt directly, with a per-shape solution search.
//
// torch.mm takes hipBLASLt's first heuristic pick.  For the engine's tall-skinny activation GEMMs
// (rows = batch x steps, up to 819200) and its long-K weight gradients that pick is often not the
// fastest solution: across all solutions, config #5's encoder GEMMs run 5-27 % faster
// (tools/micro/hipblaslt_probe.cpp, profiles/r4/ab/blt_gemm.md).  blt_mm asks the library for
// its top candidates once per (layout, shape, leading dims, output dtype, beta, bias) key, times
// each on the real operands the first time the key is seen outside a stream capture, and keeps
// the fastest.  Later calls (and hipGraph captures) reuse the pick.
//
// Row-major notation, as the model issues them:  out[M,N] = beta*out + op(a) . op(b) (+ bias[N])
//   a: [M,K] (ta = false) or [K,M] stored (ta = true);  b: [K,N] (tb = false) or [N,K] (tb = true)
//   bf16 operands, fp32 accumulate, fp32 or bf16 out; every operand row-contiguous (stride(1) == 1)
//   with its own leading dimension, so row slices of bigger buffers go straight in.
// hipBLASLt is column-major: the call computes out^T[N,M] = op(b)^T-as-stored . op(a)^T-as-stored.
//
// One workspace per HIP stream (the row-group and deferred-gradient streams run GEMMs concurrently),
// allocated on the first eager call on that stream; a stream first seen inside a capture (the
// capture stream of torch.cuda.graph) takes one of the spares allocated on the first call.  No
// solution ever runs with a workspace smaller than it reports needing (a null workspace under
// capture faulted the GPU in round 4: profiles/r4/ab/blt_gemm.md).  Workspaces come from torch's
// caching allocator (an allocation failure is torch.cuda.OutOfMemoryError, which `--batch auto`
// steps down from) and are never freed: captured graphs keep their pointers.  The count is bounded
// by torch's stream pool (32 streams per priority and device, recycled round-robin, so the same
// handles come back); TSAMD_BLT_MAX_WS (72) caps it regardless, later streams then running only
// workspace-free solutions (the key records which).
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

using at::Tensor;

namespace {

#define BLT_CK(x)                                                                                       \
  do {                                                                                                  \
    auto _s = (x);                                                                                      \
    TORCH_CHECK((int)_s == 0, "blt_mm: ", #x, " failed with status ", (int)_s);                         \
  } while (0)

constexpr size_t kWorkspace = 128ull << 20;

struct Key {
  bool ta, tb;
  int64_t M, N, K, lda, ldb, ldc;
  int out_bf16, beta_nz, bias_kind;  // bias_kind: 0 none, 1 fp32, 2 bf16
  bool ws, det;                      // det: deterministic mode (first fitting pick, never timed)
  auto tie() const { return std::tie(ta, tb, M, N, K, lda, ldb, ldc, out_bf16, beta_nz, bias_kind, ws, det); }
  bool operator<(const Key& o) const { return tie() < o.tie(); }
};

struct Pick {
  hipblasLtMatmulAlgo_t algo;
  size_t ws;
  bool tuned;
  float us;       // the pick's time when tuned
  float heur_us;  // the first heuristic's time when tuned
  int n_cand;
};

struct State {
  std::mutex mu;
  hipblasLtHandle_t handle = nullptr;
  std::map<Key, Pick> picks;
  std::map<hipStream_t, void*> ws;
  std::vector<Tensor> owned;  // every workspace (torch caching allocator), kept for the process
  std::vector<void*> spare;   // allocated eagerly, handed to streams first seen inside a capture
  bool spares_made = false;
  int64_t tuned = 0, calls = 0;
};

State& st() {
  static State* s = new State();  // never destroyed: the library may unload after the HIP runtime
  return *s;
}

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  BLT_CK(hipStreamIsCapturing(s, &cs));
  return cs != hipStreamCaptureStatusNone;
}

int env_int(const char* n, int d) {
  const char* v = std::getenv(n);
  return v && *v ? std::atoi(v) : d;
}

void* new_workspace(State& S, const Tensor& like) {
  S.owned.push_back(at::empty({(int64_t)kWorkspace}, like.options().dtype(at::kByte)));
  return S.owned.back().data_ptr();
}

struct Desc {
  hipblasLtMatmulDesc_t mm = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  ~Desc() {
    if (la) hipblasLtMatrixLayoutDestroy(la);
    if (lb) hipblasLtMatrixLayoutDestroy(lb);
    if (lc) hipblasLtMatrixLayoutDestroy(lc);
    if (mm) hipblasLtMatmulDescDestroy(mm);
  }
};

// hipBLASLt "A" is the model's b, hipBLASLt "B" is the model's a (column-major transpose).
void make_desc(Desc& d, const Key& k, const void* bias_ptr) {
  BLT_CK(hipblasLtMatmulDescCreate(&d.mm, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t opa = k.tb ? HIPBLAS_OP_T : HIPBLAS_OP_N, opb = k.ta ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  BLT_CK(hipblasLtMatmulDescSetAttribute(d.mm, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)));
  BLT_CK(hipblasLtMatmulDescSetAttribute(d.mm, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)));
  if (k.bias_kind) {
    hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_BIAS;
    hipDataType bt = k.bias_kind == 1 ? HIP_R_32F : HIP_R_16BF;
    BLT_CK(hipblasLtMatmulDescSetAttribute(d.mm, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)));
    BLT_CK(hipblasLtMatmulDescSetAttribute(d.mm, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
    BLT_CK(hipblasLtMatmulDescSetAttribute(d.mm, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias_ptr, sizeof(bias_ptr)));
  }
  // model b: [K,N] stored = col-major [N,K] (ld ldb); transposed: [N,K] stored = col-major [K,N]
  if (!k.tb) BLT_CK(hipblasLtMatrixLayoutCreate(&d.la, HIP_R_16BF, k.N, k.K, k.ldb));
  else BLT_CK(hipblasLtMatrixLayoutCreate(&d.la, HIP_R_16BF, k.K, k.N, k.ldb));
  if (!k.ta) BLT_CK(hipblasLtMatrixLayoutCreate(&d.lb, HIP_R_16BF, k.K, k.M, k.lda));
  else BLT_CK(hipblasLtMatrixLayoutCreate(&d.lb, HIP_R_16BF, k.M, k.K, k.lda));
  BLT_CK(hipblasLtMatrixLayoutCreate(&d.lc, k.out_bf16 ? HIP_R_16BF : HIP_R_32F, k.N, k.M, k.ldc));
}

hipblasStatus_t run(State& S, const Desc& d, const hipblasLtMatmulAlgo_t* algo, const void* A, const void* B,
                    float beta, void* C, void* ws, size_t wsb, hipStream_t s) {
  float alpha = 1.f;
  return hipblasLtMatmul(S.handle, d.mm, &alpha, B, d.la, A, d.lb, &beta, C, d.lc, C, d.lc, algo, ws, wsb, s);
}

float time_us(State& S, const Desc& d, const hipblasLtMatmulAlgo_t* algo, const void* A, const void* B, float beta,
              void* C, void* ws, size_t wsb, hipStream_t s) {
  if (run(S, d, algo, A, B, beta, C, ws, wsb, s) != HIPBLAS_STATUS_SUCCESS) return -1.f;  // warm
  hipEvent_t e0, e1;
  BLT_CK(hipEventCreate(&e0));
  BLT_CK(hipEventCreate(&e1));
  BLT_CK(hipEventRecord(e0, s));
  run(S, d, algo, A, B, beta, C, ws, wsb, s);
  BLT_CK(hipEventRecord(e1, s));
  BLT_CK(hipEventSynchronize(e1));
  float ms = 0.f;
  BLT_CK(hipEventElapsedTime(&ms, e0, e1));
  int reps = ms < 0.05f ? 10 : (ms < 0.5f ? 4 : 2);
  BLT_CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i) run(S, d, algo, A, B, beta, C, ws, wsb, s);
  BLT_CK(hipEventRecord(e1, s));
  BLT_CK(hipEventSynchronize(e1));
  BLT_CK(hipEventElapsedTime(&ms, e0, e1));
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return ms * 1000.f / reps;
}

void check_operand(const Tensor& t, const char* name, bool out) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 2, "blt_mm: ", name, " must be a 2-D GPU tensor");
  TORCH_CHECK(out ? (t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16) : t.scalar_type() == at::kBFloat16,
              "blt_mm: ", name, " has dtype ", t.scalar_type());
  TORCH_CHECK(t.stride(1) == 1 && (t.size(0) <= 1 || t.stride(0) >= t.size(1)), "blt_mm: ", name,
              " must be row-contiguous, strides ", t.strides());
}

void blt_mm(const Tensor& a, const Tensor& b, const Tensor& out, bool ta, bool tb, double beta,
            const std::optional<Tensor>& bias) {
  check_operand(a, "a", false);
  check_operand(b, "b", false);
  check_operand(out, "out", true);
  const int64_t M = ta ? a.size(1) : a.size(0), K = ta ? a.size(0) : a.size(1);
  const int64_t N = tb ? b.size(0) : b.size(1), Kb = tb ? b.size(1) : b.size(0);
  TORCH_CHECK(K == Kb && out.size(0) == M && out.size(1) == N, "blt_mm: shape mismatch a ", a.sizes(), " ta ", ta,
              " b ", b.sizes(), " tb ", tb, " out ", out.sizes());
  TORCH_CHECK(M > 0 && N > 0 && K > 0, "blt_mm: empty problem");
  int bias_kind = 0;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->is_cuda() && bias->is_contiguous() && bias->numel() == N, "blt_mm: bias must hold N elements");
    TORCH_CHECK(bias->scalar_type() == at::kFloat || bias->scalar_type() == at::kBFloat16, "blt_mm: bias dtype");
    bias_kind = bias->scalar_type() == at::kFloat ? 1 : 2;
  }
  auto lds = [](const Tensor& t) { return t.size(0) <= 1 ? std::max<int64_t>(t.size(1), 1) : t.stride(0); };
  hipStream_t s = c10::hip::getCurrentHIPStream().stream();
  State& S = st();
  std::lock_guard<std::mutex> g(S.mu);
  if (!S.handle) BLT_CK(hipblasLtCreate(&S.handle));
  const bool cap = capturing(s);
  if (!cap && !S.spares_made) {
    S.spares_made = true;
    // spare workspaces for the capture streams (torch.cuda.graph captures on a stream of its
    // own): no allocation can happen inside a capture, and a solution that needs a workspace
    // must never get a null one
    for (int i = 0; i < std::max(0, env_int("TSAMD_BLT_SPARE_WS", 4)); ++i) S.spare.push_back(new_workspace(S, out));
  }
  void* ws = nullptr;
  auto wit = S.ws.find(s);
  if (wit != S.ws.end()) {
    ws = wit->second;
  } else if (!cap && (int)S.ws.size() < env_int("TSAMD_BLT_MAX_WS", 72)) {
    ws = new_workspace(S, out);
    S.ws[s] = ws;
  } else if (cap && !S.spare.empty()) {
    ws = S.spare.back();
    S.spare.pop_back();
    S.ws[s] = ws;
  }
  const size_t wsb = ws ? kWorkspace : 0;
  const bool det = env_int("TSAMD_DETERMINISTIC", 0) != 0;
  Key k{ta, tb, M, N, K, lds(a), lds(b), lds(out), out.scalar_type() == at::kBFloat16, beta != 0.0, bias_kind, ws != nullptr,
        det};
  const void* bias_ptr = bias_kind ? bias->data_ptr() : nullptr;
  Desc d;
  make_desc(d, k, bias_ptr);
  // TSAMD_BLT_TRACE=1: every call's key on stderr, a stream sync after every eager call and
  // candidate, so a faulting GEMM names itself
  static const bool trace = env_int("TSAMD_BLT_TRACE", 0) != 0;
  if (trace) {
    std::fprintf(stderr, "[blt] ta %d tb %d M %ld N %ld K %ld ld %ld %ld %ld out_bf16 %d beta %g bias %d ws %d cap %d "
                 "a %p b %p out %p stream %p\n", (int)ta, (int)tb, (long)M, (long)N, (long)K, (long)k.lda, (long)k.ldb,
                 (long)k.ldc, k.out_bf16, beta, bias_kind, (int)(ws != nullptr), (int)cap, a.data_ptr(), b.data_ptr(),
                 out.data_ptr(), (void*)s);
    std::fflush(stderr);
  }
  ++S.calls;
  auto it = S.picks.find(k);
  if (it == S.picks.end()) {
    hipblasLtMatmulPreference_t pref;
    BLT_CK(hipblasLtMatmulPreferenceCreate(&pref));
    uint64_t w64 = wsb;
    BLT_CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &w64, sizeof(w64)));
    // deterministic mode: the library's first fitting pick, so a run's GEMMs do not depend on
    // another run's timings (bit-reproducible across processes, not only within one)
    const bool tune = !cap && env_int("TSAMD_BLT_TUNE", 1) != 0 && !det;
    const int want = tune ? std::max(1, env_int("TSAMD_BLT_CANDIDATES", 24)) : 8;
    std::vector<hipblasLtMatmulHeuristicResult_t> hr(want);
    int got = 0;
    BLT_CK(hipblasLtMatmulAlgoGetHeuristic(S.handle, d.mm, d.la, d.lb, d.lc, d.lc, pref, want, hr.data(), &got));
    hipblasLtMatmulPreferenceDestroy(pref);
    TORCH_CHECK(got > 0, "blt_mm: hipBLASLt has no solution for M=", M, " N=", N, " K=", K);
    // the first candidate whose workspace fits: the library can return solutions needing more
    // than the preference allows, and a null / short workspace is an out-of-bounds write
    int first = -1;
    for (int i = 0; i < got && first < 0; ++i)
      if (hr[i].state == HIPBLAS_STATUS_SUCCESS && hr[i].workspaceSize <= wsb && (ws || hr[i].workspaceSize == 0))
        first = i;
    TORCH_CHECK(first >= 0, "blt_mm: no hipBLASLt solution fits a ", wsb, "-byte workspace for M=", M, " N=", N,
                " K=", K);
    if (trace && (first > 0 || hr[0].workspaceSize > wsb))
      std::fprintf(stderr, "[blt] heuristic 0 needs %zu workspace bytes of %zu: candidate %d\n", hr[0].workspaceSize,
                   wsb, first);
    Pick p{hr[first].algo, hr[first].workspaceSize, false, -1.f, -1.f, got};
    if (tune && got > 1) {
      // time on a scratch output: an accumulating (beta != 0) call must not touch `out` here
      Tensor scratch = at::zeros({M, k.ldc}, out.options());
      float best = -1.f;
      for (int i = 0; i < got; ++i) {
        if (hr[i].state != HIPBLAS_STATUS_SUCCESS || hr[i].workspaceSize > wsb || (!ws && hr[i].workspaceSize)) continue;
        if (trace) {
          std::fprintf(stderr, "[blt] cand %d/%d ws %zu\n", i, got, hr[i].workspaceSize);
          std::fflush(stderr);
        }
        float t = time_us(S, d, &hr[i].algo, a.data_ptr(), b.data_ptr(), (float)beta, scratch.data_ptr(), ws, wsb, s);
        if (trace) BLT_CK(hipStreamSynchronize(s));
        if (i == first) p.heur_us = t;
        if (t > 0.f && (best < 0.f || t < best)) {
          best = t;
          p.algo = hr[i].algo;
          p.ws = hr[i].workspaceSize;
        }
      }
      p.tuned = true;
      p.us = best;
      ++S.tuned;
    }
    it = S.picks.emplace(k, p).first;
  }
  BLT_CK(run(S, d, &it->second.algo, a.data_ptr(), b.data_ptr(), (float)beta, out.data_ptr(), ws, wsb, s));
  if (trace && !cap) BLT_CK(hipStreamSynchronize(s));
}

// [keys, tuned keys, calls] and, per tuned key, [M, N, K, ta, tb, heuristic us, pick us, candidates]
std::vector<double> blt_stats() {
  State& S = st();
  std::lock_guard<std::mutex> g(S.mu);
  std::vector<double> r{(double)S.picks.size(), (double)S.tuned, (double)S.calls};
  for (auto& kv : S.picks) {
    if (!kv.second.tuned) continue;
    const Key& k = kv.first;
    r.insert(r.end(), {(double)k.M, (double)k.N, (double)k.K, (double)k.ta, (double)k.tb, kv.second.heur_us,
                       kv.second.us, (double)kv.second.n_cand});
  }
  return r;
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(tsamd, m) {
  m.def("blt_mm", &blt_mm);
  m.def("blt_stats", &blt_stats);
}
