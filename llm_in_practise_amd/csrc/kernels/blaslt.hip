// Direct hipBLASLt calls for the frozen-base training GEMMs (host code only).
//
// Why not torch.addmm: a 2-D residual makes aten copy the residual into the output and run the
// GEMM with beta = 1 (one extra 16 MB copy per o_proj / down_proj call, 72 per Qwen3-8B step);
// hipBLASLt itself takes C and D as separate matrices.  The plan cache also lets a shape pick its
// kernel from the measured time of the heuristic's top candidates IN the running step (cold
// weights just written by the NF4 dequant, the real L2 / MALL state; timed with events read back on
// later calls, so the host never waits) instead of the heuristic's
// first choice or an isolated-loop tuner (profiles/tunableop_ab.txt: isolated tuning predicted
// 10-20 % per GEMM and delivered 0.8 % in the step).
//
// Row-major Y[M,N] = X[M,K]·W[N,K]ᵀ is column-major Yᵀ = op(W)·X with op = T ("TN");
// dX[M,K] = dY[M,N]·W[N,K] is column-major dXᵀ = W(col-major K×N)·dYᵀ ("NN").
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

namespace {

#define LT_OK(x)                                                                             \
  do {                                                                                       \
    hipblasStatus_t s__ = (x);                                                               \
    if (s__ != HIPBLAS_STATUS_SUCCESS) {                                                     \
      fprintf(stderr, "hipBLASLt error %d at %s:%d (%s)\n", (int)s__, __FILE__, __LINE__, #x); \
      return false;                                                                          \
    }                                                                                        \
  } while (0)

using Key = std::tuple<int, int, long, long, long, long, long, long, long, int, long, long, int>;

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr, d = nullptr;
  std::vector<hipblasLtMatmulHeuristicResult_t> cand;
  std::vector<float> best;  // per-candidate best time (ms) while tuning
  std::vector<int> seen;    // timings collected per candidate
  int calls = 0, chosen = -1;
  // timings in flight: read back with hipEventQuery on later calls, never waited for (no host stall)
  struct Pending {
    int idx;
    hipEvent_t e0, e1;
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> pool;
};

hipEvent_t take_event(Plan& p) {
  if (!p.pool.empty()) {
    hipEvent_t e = p.pool.back();
    p.pool.pop_back();
    return e;
  }
  hipEvent_t e;
  hipEventCreate(&e);
  return e;
}

// fold finished timings in; choose once every candidate has tune_reps() of them
void poll_timings(Plan& p, int reps) {
  for (size_t i = 0; i < p.pending.size();) {
    Plan::Pending& t = p.pending[i];
    if (hipEventQuery(t.e1) != hipSuccess) {
      ++i;
      continue;
    }
    float ms = 0.f;
    hipEventElapsedTime(&ms, t.e0, t.e1);
    if (ms < p.best[t.idx]) p.best[t.idx] = ms;
    ++p.seen[t.idx];
    p.pool.push_back(t.e0);
    p.pool.push_back(t.e1);
    p.pending[i] = p.pending.back();
    p.pending.pop_back();
  }
  if (p.chosen >= 0) return;
  for (size_t i = 0; i < p.cand.size(); ++i)
    if (p.seen[i] < reps) return;
  int bi = 0;
  for (int i = 1; i < (int)p.cand.size(); ++i)
    if (p.best[i] < p.best[bi]) bi = i;
  p.chosen = bi;
}

hipblasLtHandle_t g_handle = nullptr;
std::map<Key, Plan> g_plans;
std::mutex g_mu;

int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

// number of heuristic candidates timed per shape (1 = the heuristic's first choice, no timing)
int n_candidates() {
  static const int n = [] { int v = env_int("LIPA_LT_CANDIDATES", 4); return v < 1 ? 1 : (v > 16 ? 16 : v); }();
  return n;
}
int tune_reps() {
  static const int n = [] { int v = env_int("LIPA_LT_REPS", 3); return v < 1 ? 1 : v; }();
  return n;
}

bool make_plan(Plan& p, bool ta, bool tb, long m, long n, long k, long lda, long ldb, long ldc, int batch,
               long sa, long sb, long sc, size_t ws) {
  const hipDataType dt = HIP_R_16BF;
  LT_OK(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F));
  hipblasOperation_t opa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, opb = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  LT_OK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &opa, sizeof(opa)));
  LT_OK(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &opb, sizeof(opb)));
  LT_OK(hipblasLtMatrixLayoutCreate(&p.a, dt, ta ? k : m, ta ? m : k, lda));
  LT_OK(hipblasLtMatrixLayoutCreate(&p.b, dt, tb ? n : k, tb ? k : n, ldb));
  LT_OK(hipblasLtMatrixLayoutCreate(&p.c, dt, m, n, ldc));
  LT_OK(hipblasLtMatrixLayoutCreate(&p.d, dt, m, n, ldc));
  if (batch > 1) {
    const int32_t bc = batch;
    const int64_t strides[3] = {sa, sb, sc};
    hipblasLtMatrixLayout_t ls[4] = {p.a, p.b, p.c, p.d};
    for (int i = 0; i < 4; ++i) {
      const int64_t st = strides[i < 3 ? i : 2];
      LT_OK(hipblasLtMatrixLayoutSetAttribute(ls[i], HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &bc, sizeof(bc)));
      LT_OK(hipblasLtMatrixLayoutSetAttribute(ls[i], HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &st, sizeof(st)));
    }
  }
  hipblasLtMatmulPreference_t pref;
  LT_OK(hipblasLtMatmulPreferenceCreate(&pref));
  const uint64_t wsb = ws;
  LT_OK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb)));
  std::vector<hipblasLtMatmulHeuristicResult_t> res(16);
  int got = 0;
  const hipblasStatus_t hs =
      hipblasLtMatmulAlgoGetHeuristic(g_handle, p.desc, p.a, p.b, p.c, p.d, pref, 16, res.data(), &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (hs != HIPBLAS_STATUS_SUCCESS || got == 0) return false;
  for (int i = 0; i < got && (int)p.cand.size() < n_candidates(); ++i)
    if (res[i].state == HIPBLAS_STATUS_SUCCESS && res[i].workspaceSize <= ws) p.cand.push_back(res[i]);
  if (p.cand.empty()) return false;
  p.best.assign(p.cand.size(), 1e30f);
  p.seen.assign(p.cand.size(), 0);
  if (p.cand.size() == 1) p.chosen = 0;
  return true;
}

}  // namespace

// D = op(A)·op(B) (+ C when C != nullptr; beta = 1), column-major, bf16 in/out, fp32 accumulate.
// tune: time the heuristic's top candidates on the first calls of the shape and keep the fastest.
// Returns false when hipBLASLt has no plan for the problem (the caller falls back).
bool lt_gemm(bool ta, bool tb, long m, long n, long k, const void* A, long lda, const void* B, long ldb,
             const void* C, void* D, long ldc, int batch, long sa, long sb, long sc, void* ws, size_t ws_bytes,
             hipStream_t st, bool tune) {
  Plan* p;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_handle && hipblasLtCreate(&g_handle) != HIPBLAS_STATUS_SUCCESS) return false;
    const Key key{ta, tb, m, n, k, lda, ldb, ldc, 0, batch, sa, sb, C != nullptr};
    auto it = g_plans.find(key);
    if (it == g_plans.end()) {
      Plan np;
      if (!make_plan(np, ta, tb, m, n, k, lda, ldb, ldc, batch, sa, sb, sc, ws_bytes)) return false;
      it = g_plans.emplace(key, np).first;
    }
    p = &it->second;
  }
  const float alpha = 1.f, beta = C ? 1.f : 0.f;
  if (p->chosen < 0 && !p->pending.empty()) {
    std::lock_guard<std::mutex> lk(g_mu);
    const int before = p->chosen;
    poll_timings(*p, tune_reps());
    if (before < 0 && p->chosen >= 0 && env_int("LIPA_LT_VERBOSE", 0))
      fprintf(stderr, "[lt] m=%ld n=%ld k=%ld b=%d C=%d: candidate %d of %zu (%.1f us; first %.1f us)\n", m, n, k,
              batch, C != nullptr, p->chosen, p->cand.size(), 1e3f * p->best[p->chosen], 1e3f * p->best[0]);
  }
  int idx = p->chosen;
  Plan::Pending timing{-1, nullptr, nullptr};
  if (idx < 0 && (!tune || (getenv("LIPA_DETERMINISTIC") && atoi(getenv("LIPA_DETERMINISTIC"))))) {
    // reproducible runs, or a shape called once per step: the heuristic's first choice, no rotation
    idx = 0;
  } else if (idx < 0) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hipStreamIsCapturing(st, &cs);
    idx = 0;   // no timing inside a graph capture
    if (cs == hipStreamCaptureStatusNone) {
      const int nc = (int)p->cand.size();
      idx = p->calls++ % nc;
      if (p->pending.size() < 64) {
        std::lock_guard<std::mutex> lk(g_mu);
        timing = {idx, take_event(*p), take_event(*p)};
        hipEventRecord(timing.e0, st);
      }
    }
  }
  const hipblasStatus_t s =
      hipblasLtMatmul(g_handle, p->desc, &alpha, A, p->a, B, p->b, &beta, C ? C : D, p->c, D, p->d,
                      &p->cand[idx].algo, ws, ws_bytes, st);
  if (s != HIPBLAS_STATUS_SUCCESS) {
    fprintf(stderr, "hipBLASLt matmul failed (%d) m=%ld n=%ld k=%ld\n", (int)s, m, n, k);
    return false;
  }
  if (timing.idx >= 0) {
    hipEventRecord(timing.e1, st);
    std::lock_guard<std::mutex> lk(g_mu);
    p->pending.push_back(timing);
  }
  return true;
}

// reset the per-shape choices (tests / A-B runs)
void lt_reset() {
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto& kv : g_plans) {
    Plan& p = kv.second;
    hipblasLtMatmulDescDestroy(p.desc);
    hipblasLtMatrixLayoutDestroy(p.a);
    hipblasLtMatrixLayoutDestroy(p.b);
    hipblasLtMatrixLayoutDestroy(p.c);
    hipblasLtMatrixLayoutDestroy(p.d);
    for (auto& t : p.pending) {
      hipEventDestroy(t.e0);
      hipEventDestroy(t.e1);
    }
    for (hipEvent_t e : p.pool) hipEventDestroy(e);
  }
  g_plans.clear();
}
