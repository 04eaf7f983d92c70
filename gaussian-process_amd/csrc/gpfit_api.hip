// gpfit_api.hip — host side of libgpfit.so: the C-ABI declared in include/gpfit.h.
//
// One context = one HIP device + one stream + device-resident training data.
// gpf_eval_batch replaces the reference's process-pool fan-out over particles
// (find_len_scales.py:73-77,102-104,133-135): non-sentinel particles are packed
// into chunks that fit HBM and every chunk is one batched factorise+score.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gpfit.h"
#include "gpf_common.hip"
#include "gpf_covariance.hip"
#include "gpf_factor.hip"
#include "gpf_persist.hip"
#include "gpf_objective.hip"
#include "gpf_predict.hip"
#include "gpf_probsurf.hip"
#include "gpf_hull.hip"
#include "gpf_kmeans.hip"

using gpf::BT;
using gpf::NTHR;
using gpf::T;

namespace {

enum ProfClass { PC_PANEL = 0, PC_DIAG = 1, PC_BUILD = 2, PC_LOSS = 3, PC_FACTOR = 4, PC_PRED = 5, PC_PREDK = 6, PC_PSURF = 7, PC_N = 8 };

constexpr int MAX_GROUPS = 4;  // particle groups factorised on concurrent streams
constexpr int GRAPH_NT_MAX = 2;  // eval batches with N <= 256 run as a replayed HIP graph
// a captured batch must never reach split_plan's hipMalloc/hipFree (splits start at nt = 4)
static_assert(GRAPH_NT_MAX < 4, "graph-captured batches must not use split-K buffers");

struct Pending {
  hipEvent_t a, b;
  int cls;
  double work;  // algorithmic flops or bytes of this launch
};

}  // namespace

struct gpf_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t sub[MAX_GROUPS] = {};  // one stream per particle group (run_factor)
  hipEvent_t fork = nullptr, join[MAX_GROUPS] = {};
  std::string err;

  // training data
  int64_t N = 0, Npad = 0;
  int d = 0, nt = 0;
  double* d_x = nullptr;
  double* d_y = nullptr;
  double* d_e = nullptr;
  std::vector<double> h_y;

  // objective grid / box
  int K = 0;
  double* d_sig = nullptr;
  double* d_exp = nullptr;
  double* d_lo = nullptr;
  double* d_hi = nullptr;
  std::vector<double> h_lo, h_hi;

  // per-chunk workspace
  int cap = 0;  // particles per chunk the workspace holds
  double* d_L = nullptr;
  double* d_U = nullptr;
  double* d_yb = nullptr;
  double* d_s2p = nullptr;
  double* d_part = nullptr;    // split-K partial products (run_factor, few tiles per launch)
  unsigned* d_cnt = nullptr;   // split-K arrival counters, one per (particle, tile), kept zero
  size_t part_cap = 0, cnt_cap = 0;
  double* d_la = nullptr;      // look-ahead partials of the next critical tiles (gpf::la_item), one tile per particle
  size_t la_cap = 0;
  double* d_pb = nullptr;      // paired block columns: the lead launch's partials, nt-1 tiles per particle (gpf::pair_slot)
  size_t pb_cap = 0;
  int* d_pstart = nullptr;     // ... and the partners' start words (gpf::pair_start_sync), PAIR_HMAX per tile
  size_t pstart_cap = 0;
  double* d_lb = nullptr;      // all-tile look-ahead pieces (gpf::lall_slot): two parities x particles x smax slots
  size_t lb_cap = 0;
  int fact_seq = 0;            // factorisations run (tags the start words)
  double* d_szp = nullptr;
  double* d_ls = nullptr;
  double* d_mu = nullptr;
  double* d_sd = nullptr;
  double* d_loss = nullptr;
  int* d_info = nullptr;
  int* d_flag = nullptr;  // per particle: last diagonal block published in the running launch (early_diag)
  int* d_cflag = nullptr;  // per particle: last diagonal block reduced by a SYRK workgroup (defer_syrk); reset by k_build_cov
  int* d_pst = nullptr;    // the persistent factorisation's counters (gpf::PState: 3 x cap x nt, heads, abort); reset by k_build_cov
  int ncu = 0;             // compute units of the device (the persistent launch's grid: two workgroups per CU)
  // gpf_predict's query-chunk buffers, kept between calls (grow-only; freed with the work buffers)
  double *p_xf = nullptr, *p_ks = nullptr, *p_vsq = nullptr, *p_mu = nullptr, *p_sd = nullptr;
  double *p_hx = nullptr, *p_hout = nullptr;  // pinned staging: query coordinates, (mu, sd)
  double* p_vz = nullptr;                      // per row tile of V = U K_s: V^T z partials of mu (gpf::k_predict_vsq)
  int64_t p_cols = 0, p_np = 0;
  int p_d = 0, p_nt = 0;
  // gpf_prob_surface's row-chunk buffers, kept between calls like the prediction's
  double *s_t = nullptr, *s_cmp = nullptr, *s_y = nullptr, *s_p = nullptr;
  double4* s_info = nullptr;
  int* s_ok = nullptr;
  int64_t s_rows = 0;
  int s_e = 0;
  int* d_hist = nullptr;
  // pinned host staging for the per-batch transfers (async DMA, capturable in graphs)
  double* h_ls = nullptr;
  double* h_loss = nullptr;
  int* h_info = nullptr;
  // KMeans subsample (gpf_kmeans_set / gpf_kmeans_step): the centred points and the per-step buffers
  double *km_x = nullptr, *km_c = nullptr, *km_dist = nullptr, *km_sums = nullptr, *km_cnt = nullptr;
  int* km_lab = nullptr;
  int64_t km_n = 0;
  int km_d = 0, km_kcap = 0, km_cd = 0;  // km_cd: the d the centre buffers were sized for
  // last convex-hull grid (gpf_hull_fill -> gpf_hull_fetch)
  std::vector<double> hull_rows;
  int hull_d = 0;
  // small-problem path: one captured graph per batch size (launch-latency bound regime)
  std::vector<std::pair<int, hipGraphExec_t>> graphs;

  // profiling
  bool prof = false;
  unsigned long long* d_clk = nullptr;  // shader-clock probe of the factor kernels (gpf::ClockSpan), profiling only
  double bench_sclk = 0.0;              // shader clock (MHz) of the last gpf_mfma_peak / gpf_gemm_bench
  double acc[PC_N][3] = {};  // ms, launches, work
  double evals = 0;
  std::vector<Pending> pend;
  std::vector<hipEvent_t> pool;
};

#define GPF_HIP(ctx, expr)                                                                   \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) {                                                                  \
      (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(_e);                        \
      return GPF_HIP_ERROR;                                                                  \
    }                                                                                        \
  } while (0)

static int bad_arg(gpf_ctx* c, const char* m) {
  c->err = m;
  return GPF_BAD_ARG;
}

static hipEvent_t take_event(gpf_ctx* c) {
  if (!c->pool.empty()) {
    hipEvent_t e = c->pool.back();
    c->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Launch helper: brackets the launch with events when profiling is on.
template <typename F>
static int launch_on(gpf_ctx* c, hipStream_t st, int cls, double work, F f) {
  hipEvent_t a = nullptr, b = nullptr;
  if (c->prof) {
    a = take_event(c);
    b = take_event(c);
    if (a && b) hipEventRecord(a, st);
  }
  f();
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    c->err = std::string("kernel launch: ") + hipGetErrorString(e);
    return GPF_HIP_ERROR;
  }
  if (c->prof && a && b) {
    hipEventRecord(b, st);
    c->pend.push_back({a, b, cls, work});
  }
  return GPF_OK;
}

template <typename F>
static int launch(gpf_ctx* c, int cls, double work, F f) {
  return launch_on(c, c->stream, cls, work, f);
}

static void harvest(gpf_ctx* c) {
  for (auto& p : c->pend) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      c->acc[p.cls][0] += ms;
      c->acc[p.cls][1] += 1;
      c->acc[p.cls][2] += p.work;
    }
    c->pool.push_back(p.a);
    c->pool.push_back(p.b);
  }
  c->pend.clear();
}

static void clear_graphs(gpf_ctx* c) {
  for (auto& g : c->graphs) hipGraphExecDestroy(g.second);
  c->graphs.clear();
}

static void free_pred(gpf_ctx* c) {
  hipFree(c->p_xf); hipFree(c->p_ks); hipFree(c->p_vsq); hipFree(c->p_mu); hipFree(c->p_sd); hipFree(c->p_vz);
  hipHostFree(c->p_hx); hipHostFree(c->p_hout);
  c->p_xf = c->p_ks = c->p_vsq = c->p_mu = c->p_sd = c->p_vz = nullptr;
  c->p_hx = c->p_hout = nullptr;
  c->p_cols = c->p_np = 0;
  c->p_d = c->p_nt = 0;
}

static void free_psurf(gpf_ctx* c) {
  hipFree(c->s_t); hipFree(c->s_cmp); hipFree(c->s_y); hipFree(c->s_p); hipFree(c->s_info); hipFree(c->s_ok);
  c->s_t = c->s_cmp = c->s_y = c->s_p = nullptr;
  c->s_info = nullptr;
  c->s_ok = nullptr;
  c->s_rows = 0;
  c->s_e = 0;
}

// Device buffers of gpf_predict / gpf_prob_surface are kept for the next call unless larger
// than GPF_PREDICT_KEEP_MB (default 2048): a one-off large call must not hold HBM that would
// starve the next factorisation's or hull's allocations
static double keep_bytes() {
  double keep_mb = 2048.0;
  if (const char* e = getenv("GPF_PREDICT_KEEP_MB")) keep_mb = atof(e);
  return keep_mb * 1048576.0;
}

static void free_work(gpf_ctx* c) {
  clear_graphs(c);
  free_pred(c);
  free_psurf(c);
  hipHostFree(c->h_ls); hipHostFree(c->h_loss); hipHostFree(c->h_info);
  c->h_ls = c->h_loss = nullptr;
  c->h_info = nullptr;
  hipFree(c->d_L); hipFree(c->d_U); hipFree(c->d_yb); hipFree(c->d_s2p); hipFree(c->d_szp);
  hipFree(c->d_ls); hipFree(c->d_mu); hipFree(c->d_sd); hipFree(c->d_loss); hipFree(c->d_info);
  hipFree(c->d_hist);
  hipFree(c->d_flag);
  c->d_flag = nullptr;
  hipFree(c->d_cflag);
  c->d_cflag = nullptr;
  hipFree(c->d_pst);
  c->d_pst = nullptr;
  hipFree(c->d_part); hipFree(c->d_cnt);
  c->d_part = nullptr;
  c->d_cnt = nullptr;
  c->part_cap = c->cnt_cap = 0;
  hipFree(c->d_la);
  c->d_la = nullptr;
  c->la_cap = 0;
  hipFree(c->d_pb);
  c->d_pb = nullptr;
  c->pb_cap = 0;
  hipFree(c->d_pstart);
  c->d_pstart = nullptr;
  c->pstart_cap = 0;
  hipFree(c->d_lb);
  c->d_lb = nullptr;
  c->lb_cap = 0;
  c->d_L = c->d_U = c->d_yb = c->d_s2p = c->d_szp = c->d_ls = c->d_mu = c->d_sd = c->d_loss = nullptr;
  c->d_info = nullptr;
  c->d_hist = nullptr;
  c->cap = 0;
}

static size_t bytes_per_particle(const gpf_ctx* c) {
  const size_t np = (size_t)c->Npad;
  // (+ the paired block columns' partial slots, nt-1 tiles, allocated when a factorisation pairs)
  return 2 * np * np * 8 + (2 * (size_t)c->nt * np + 3 * np) * 8 + (size_t)(c->K + 1) * 4 + 64 * 8 + 8 +
         (size_t)std::max(c->nt - 1, 0) * T * T * 8;
}

// Chunk capacity from free HBM (GPF_MAX_CHUNK caps it, GPF_MEM_FRACTION scales the budget).
static int ensure_work(gpf_ctx* c, int want) {
  if (want <= c->cap) return GPF_OK;
  free_work(c);
  size_t fr = 0, tot = 0;
  GPF_HIP(c, hipMemGetInfo(&fr, &tot));
  double frac = 0.85;
  if (const char* s = getenv("GPF_MEM_FRACTION")) frac = atof(s);
  const size_t per = bytes_per_particle(c);
  long long fit = (long long)((double)fr * frac / (double)per);
  if (const char* s = getenv("GPF_MAX_CHUNK")) fit = std::min<long long>(fit, atoll(s));
  if (fit < 1) {
    c->err = "not enough device memory for one particle at N=" + std::to_string(c->N);
    return GPF_HIP_ERROR;
  }
  const int cap = (int)std::min<long long>(want, fit);
  const size_t np = (size_t)c->Npad;
  GPF_HIP(c, hipMalloc(&c->d_L, (size_t)cap * np * np * 8));
  GPF_HIP(c, hipMalloc(&c->d_U, (size_t)cap * np * np * 8));
  GPF_HIP(c, hipMalloc(&c->d_yb, (size_t)cap * np * 8));
  GPF_HIP(c, hipMalloc(&c->d_s2p, (size_t)cap * c->nt * np * 8));
  GPF_HIP(c, hipMalloc(&c->d_szp, (size_t)cap * c->nt * np * 8));
  GPF_HIP(c, hipMalloc(&c->d_ls, (size_t)cap * std::max(c->d, 1) * 8));
  GPF_HIP(c, hipMalloc(&c->d_mu, (size_t)cap * np * 8));
  GPF_HIP(c, hipMalloc(&c->d_sd, (size_t)cap * np * 8));
  GPF_HIP(c, hipMalloc(&c->d_loss, (size_t)cap * 8));
  GPF_HIP(c, hipMalloc(&c->d_info, (size_t)cap * 4));
  GPF_HIP(c, hipMalloc(&c->d_flag, (size_t)cap * 4));  // reset by k_build_cov at every factorisation
  GPF_HIP(c, hipMalloc(&c->d_cflag, (size_t)cap * 4));  // likewise
  GPF_HIP(c, hipMalloc(&c->d_pst, ((size_t)3 * cap * c->nt + 16) * 4));  // likewise (persistent factorisation)
  GPF_HIP(c, hipMalloc(&c->d_hist, (size_t)cap * (c->K + 1) * 4));
  // on the library stream: the legacy null stream does not order against our non-blocking streams
  GPF_HIP(c, hipMemsetAsync(c->d_hist, 0, (size_t)cap * (c->K + 1) * 4, c->stream));  // k_score re-zeroes what it read
  GPF_HIP(c, hipHostMalloc((void**)&c->h_ls, (size_t)cap * std::max(c->d, 1) * 8, hipHostMallocDefault));
  GPF_HIP(c, hipHostMalloc((void**)&c->h_loss, (size_t)cap * 8, hipHostMallocDefault));
  GPF_HIP(c, hipHostMalloc((void**)&c->h_info, (size_t)cap * 4, hipHostMallocDefault));
  c->cap = cap;
  return GPF_OK;
}

// Particle groups factorised on concurrent streams (GPF_GROUPS overrides): they fill the tail
// of each dependent block-column launch with another group's tiles. Measured on MI355X
// (profiles/r1/groups_ab.txt, profiles/r2/groups_stagger_ab.txt): 2 groups +4.6% at N=4096 P=32
// (config D's share of one GPU), +1.7% at N=4096 P=64 (config C, round 2: 1303 -> 1324
// evals/s, same box), -19% at N=1024 P=32, 4 groups worse everywhere. Default: 2 groups for
// chunks with at least 16 block columns, else 1. (With concurrent groups the per-launch times
// overlap, so bench.py rates the whole factorisation phase instead: no gaps or overlap counted.)
// Persistent factorisation (gpf::k_factor, gpf_persist.hip) for slot-bound schedules with many
// block columns: more tiles per block column than the 512 workgroup slots and nt >= 64 (config
// E's per-GPU share: 22.2-22.3 vs 22.0 evals/s, 0.945 vs 0.937 of the FP64 ceiling at the clock
// the chip held). At nt = 32 (configs C, D) the per-block-column launches on two group streams
// stay faster: 1344-1368 vs 1310-1331 evals/s — per clock the two are within 0.5%, but the chip
// holds ~40 MHz less under the persistent launch (profiles/r4/ab_persist_clock.txt,
// ab_r4g_summary.txt). B-like launches (fewer tiles than slots) lose 24% (no early diagonal
// factor in it). GPF_PERSIST = 0/1 overrides.
static bool persist_on(int pc, int nt) {
  bool on = (long long)pc * (nt - 1) > 512 && nt >= 64;
  if (const char* s = getenv("GPF_PERSIST")) on = atoi(s) != 0;
  return on && nt >= 3 && pc >= 2;  // (a single particle — the prediction — keeps its split launches)
}

static int num_groups(int pc, int nt) {
  if (persist_on(pc, nt)) return 1;  // one launch over every particle
  int g = nt >= 16 ? 2 : 1;
  if (const char* s = getenv("GPF_GROUPS")) g = atoi(s);
  g = std::max(1, std::min(g, MAX_GROUPS));
  while (g > 1 && pc / g < 8) --g;  // keep >= 8 particles (one per XCD) per group
  return g;
}

// Particles per XCD dispatch group of k_step (see gpf::step_tile); GPF_STEP_GROUP
// overrides, 0 = particle fastest over the whole launch.
static int step_group(int pc) {
  int g = 0;
  if (const char* s = getenv("GPF_STEP_GROUP")) g = atoi(s);
  return std::max(0, std::min(g, pc / 8));
}

// Split-K factor of the block-column launches: launches with at most 64 tiles (a single
// particle: the prediction path) cut every tile's GEMM into S depth ranges (gpf::flat_piece), S
// filling ~512 workgroup slots. Measured (profiles/r1/split_k_ab.txt): single-particle factor at
// N=4096 11.3 -> 9.9 ms with S=16 (7.4 ms since the partials are stored write-through, with no
// release fence); config B (224 tiles, S=2) 21.3k -> 14.3k evals/s with the fence, hence the
// threshold. At most 8 pieces since round 2 (with the split-K reduction tree and the early
// diagonal factor): an L tile's depth is 8J 16-deep chunks, so 8 pieces are always even while
// 16 leave odd-J tiles uneven and J = 1 tiles with empty pieces — single-particle factor at
// N=4096 4.17 -> 3.90 ms, N=2048 equal, N=8192 already 8 (512/63), S=16 there 16.4 vs 13.5 ms
// (profiles/r2/predict_splitk_ab.txt). GPF_SPLIT_K overrides (1 = off). Not for tiny problems (nt < 4).
static int split_k(int tiles, int nt) {
  int S = (nt >= 4 && tiles <= 64) ? std::max(1, std::min(8, 512 / std::max(1, tiles))) : 1;
  if (const char* s = getenv("GPF_SPLIT_K")) S = std::max(1, std::min(32, atoi(s)));
  if (nt < 4) S = 1;
  return S;
}

// Chunk target of launch J under the all-tile split (gpf::split_all_pieces): the launch's GEMM
// depth (pc particles, every tile) spread over `slots` workgroups of about equal work, one per CU
// (a slot per particle is kept for the diagonal workgroups — also without the early diagonal
// factor, so that both schedules sum the same pieces and stay bitwise equal: a piece that shares
// the diagonal factor's CU slows its dependent chain; two pieces per CU run at half rate each),
// with pieces of at least
// GPF_SPLIT_K_MINCH (4) 16-deep chunks. A fixed S pieces per tile (rounds 1-2) gave every tile
// the same piece count, so the deepest tiles — the critical tile I = J+1 among them — had the
// longest pieces and, from J ~ 10 on, ended the launch after the diagonal factor.
// GPF_SPLIT_K_SLOTS overrides the workgroup budget (256).
static int split_all_target(int pc, int nt, int J) {
  int slots = 256, minch = 4;
  if (const char* e = getenv("GPF_SPLIT_K_SLOTS")) slots = std::max(1, atoi(e));
  if (const char* e = getenv("GPF_SPLIT_K_MINCH")) minch = std::max(1, atoi(e));
  const int budget = std::max(1, slots - pc);
  long long tot = 0;
  for (int w = 0; w < nt - 1; ++w) tot += gpf::split_all_chunks(J, w, nt);
  const int cap = std::max(1, J * T / gpf::DL_KC);  // every tile in one piece from here on
  auto wgs = [&](int tgt) {
    long long n = 0;
    for (int w = 0; w < nt - 1; ++w) n += gpf::split_all_pieces(J, w, nt, tgt);
    return pc * n;
  };
  // smallest target >= the even share whose pieces fit the budget (the count falls with tgt)
  int lo = (int)std::min<long long>(cap, std::max<long long>(minch, (pc * tot + budget - 1) / budget)), hi = cap;
  while (lo < hi) {
    const int mid = (lo + hi) / 2;
    if (wgs(mid) <= budget) hi = mid;
    else lo = mid + 1;
  }
  const int tgt = lo;
  return std::min(tgt, cap);
}

// Early diagonal factor (gpf::k_step<SPLIT, 1>, gpf_factor.hip) for factorisations whose launches
// leave workgroup slots idle: there the launch time is the critical tile's chain, and moving the
// diagonal factor of block J to the start of launch J, beside the GEMMs, takes it off that chain
// (same-box A/B, gpurun_out r2i: config B, N=1024 P=32, 23.1k -> 29.2k evals/s; N=2048 P=32
// +5%; the single-particle prediction factor 7.1 -> 6.0 ms). Launches with more tiles than
// slots are bound by the slot load instead, and their tiles would wait for the flag in the first
// block columns (config C -0.7%, config D's 32-particle share -0.3%, E neutral), so they keep the
// fused factor. pc: the particles of all concurrent groups. GPF_EARLY_DIAG = 0/1 overrides.
// The all-tile split always runs it (its flat finish, gpf::flat_piece, waits for the diagonal block
// inside the launch): GPF_EARLY_DIAG=0 does not apply there.
static bool split_all_on(int pc, int nt) {
  const int ng = num_groups(pc, nt);
  return split_k(((pc + ng - 1) / ng) * (nt - 1), nt) > 1;
}
static bool early_diag(int pc, int nt) {
  bool on = (long long)pc * (nt - 1) <= 512;
  if (const char* s = getenv("GPF_EARLY_DIAG")) on = atoi(s) != 0;
  return (on || split_all_on(pc, nt)) && nt > 1;
}

// Deferred diagonal update (gpf::syrk_item; see gpf::step_decode) for every factorisation without
// the all-tile split. GPF_DEFER_SYRK = 0 restores the per-tile look-ahead (A/B knob).
static bool defer_syrk() {
  bool on = true;
  if (const char* s = getenv("GPF_DEFER_SYRK")) on = atoi(s) != 0;
  return on;
}

// Look-ahead of the critical tile (gpf::la_item) for launches with the early diagonal factor and
// no split: launch J (1 <= J <= nt-3) also runs the first ~7/16 of the next critical tile's GEMM
// (on its SYRK workgroups), and launch J+1's critical tile continues from there. There the
// launch's chain was that tile's depth-128J GEMM once it outgrew the diagonal factor (config B
// from J = 4): same box, B 33.8k -> 36.1k evals/s, launch spans 743 -> 687 us
// (profiles/r3s2/ab_lookahead_B.txt).
// Slot-bound launches (config C, the fused factor) gain nothing from moving work between launches.
// GPF_LOOKAHEAD = 0/1 overrides.
static bool look_ahead(int pc, int nt) {
  bool on = early_diag(pc, nt);
  if (const char* s = getenv("GPF_LOOKAHEAD")) on = atoi(s) != 0;
  return on && nt >= 4;
}

// Reordered dispatch of early-diagonal launches with SYRK workgroups (gpf::step_decode ro): the
// diagonal factors get their CUs alone. GPF_REORDER = 0/1 overrides.
static bool reorder_on() {
  bool on = true;
  if (const char* s = getenv("GPF_REORDER")) on = atoi(s) != 0;
  return on;
}

// Paired block columns (gpf::pair_decode; lead launch J streams each tile's panel once for block
// columns J and J+1, the follow launch J+1 finishes from the partials) for the fused-diagonal
// schedule without split: slot-bound launches (configs C, D) whose particle groups are multiples of 8
// (one particle per XCD in every group of 8, so a tile and its partner share an XCD) and nt >= 4.
// GPF_PAIR = 0/1 overrides.
static bool pair_on() {
  bool on = false;
  if (const char* s = getenv("GPF_PAIR")) on = atoi(s) != 0;
  return on;
}

// All-tile look-ahead in pieces (gpf::lall_decode) for the early-diagonal launches without split
// (config B: fewer tiles than workgroup slots, launches bound by their deepest tile), from launch
// GPF_LA_ALL_FROM on (default nt-2: the last launch, whose deepest U tile is the factorisation's
// longest item, consumes them: config B 41.5-41.7k -> 42.4k evals/s; from launch 1 on, or nt-3, the
// producing launches grow by more than the consumers shrink: 35-39k; profiles/r6/
// ab_B_lookahead_pieces.txt). GPF_LA_ALL = 0/1 overrides. In the launches it covers it replaces the
// critical-tile look-ahead (GPF_LOOKAHEAD) and the reordered dispatch.
static bool lall_on() {
  bool on = true;
  if (const char* s = getenv("GPF_LA_ALL")) on = atoi(s) != 0;
  return on;
}
// piece size in 128-blocks (GPF_LA_ALL_PB, 1..4) and the pieces ahead of the tiles (GPF_LA_ALL_FIRST)
static int lall_pb() {
  int pb = 1;
  if (const char* s = getenv("GPF_LA_ALL_PB")) pb = std::max(1, std::min(4, atoi(s)));
  return pb;
}
// the first launch that produces pieces (GPF_LA_ALL_FROM; default nt-2: only the last launch, whose
// deepest U tile is the longest item of the factorisation, consumes them; negative: counted from nt)
static int lall_from(int nt) {
  int j = -2;
  if (const char* s = getenv("GPF_LA_ALL_FROM")) j = atoi(s);
  return std::max(1, j < 0 ? nt + j : j);
}
static bool lall_first() {
  bool on = true;
  if (const char* s = getenv("GPF_LA_ALL_FIRST")) on = atoi(s) != 0;
  return on;
}
// (the pieces per particle and launch grow as nt J / 2: the look-ahead is for short factorisations)
constexpr int LALL_NT_MAX = 32;
static int lall_smax(int nt) {
  int m = 1;
  for (int J = 0; J < nt; ++J) m = std::max(m, gpf::lall_total(J, nt, lall_pb()));
  return m;
}

// Bound of the early-diagonal hand-off spin (gpf::wait_diag, polls of ~1 us): ~2 s by default;
// GPF_WAIT_SPINS lowers it to exercise the timeout report (tests/test_gpu.py).
static int wait_spins() {
  int n = 1 << 21;
  if (const char* s = getenv("GPF_WAIT_SPINS")) n = std::max(0, atoi(s));
  return n;
}

// Dynamic LDS that keeps a k_step launch at one workgroup per CU (its static LDS plus this exceeds
// half of the CU's 160 KiB): GPF_STEP_1PERCU = 1 for every unsplit early-diagonal launch (A/B knob).
static unsigned one_per_cu_lds(const struct StepLaunch& l);

static int ensure_split(gpf_ctx* c, int tiles, int S) {
  const size_t pb = (size_t)tiles * S * T * T * 8, cb = (size_t)tiles * gpf::split_cnt_stride(c->nt) * 4;
  if (pb > c->part_cap) {
    clear_graphs(c);  // captured graphs hold the old pointers
    hipFree(c->d_part);
    c->d_part = nullptr;
    c->part_cap = 0;
    GPF_HIP(c, hipMalloc(&c->d_part, pb));
    c->part_cap = pb;
  }
  if (cb > c->cnt_cap) {
    clear_graphs(c);
    hipFree(c->d_cnt);
    c->d_cnt = nullptr;
    c->cnt_cap = 0;
    GPF_HIP(c, hipMalloc(&c->d_cnt, cb));
    // on the library stream (the null stream would not order against it); the finishing
    // workgroups re-zero what they used
    GPF_HIP(c, hipMemsetAsync(c->d_cnt, 0, cb, c->stream));
    c->cnt_cap = cb;
  }
  return GPF_OK;
}

// Split-K plan of a factorisation of pc particles: S (all tiles) and the largest factor any
// launch uses; the partial buffers are sized for it. run_factor calls this before it forks
// the group streams. The graph path (N <= 128 * GRAPH_NT_MAX) captures run_factor, but
// split_k never splits below nt = 4, so nothing is allocated during a capture
// (static_assert below).
static void split_sizes(int pc, int nt, int& S, int& Smax) {
  const int ng = num_groups(pc, nt);
  const int gmax = (pc + ng - 1) / ng;
  S = split_k(gmax * (nt - 1), nt);
  Smax = S;
  if (S > 1) {  // the all-tile split: slots for the most pieces any tile gets
    Smax = 1;
    for (int g = 0; g < ng; ++g) {  // (the target depends on the group's particle count)
      const int gc = (int)((long long)pc * (g + 1) / ng) - (int)((long long)pc * g / ng);
      for (int J = 1; J < nt; ++J) {
        const int tgt = split_all_target(gc, nt, J);
        for (int w = 0; w < nt - 1; ++w) Smax = std::max(Smax, gpf::split_all_pieces(J, w, nt, tgt));
      }
    }
    Smax = std::max(Smax, 2);
  }
}

static int split_plan(gpf_ctx* c, int pc, int& S, int& Smax) {
  split_sizes(pc, c->nt, S, Smax);
  return Smax > 1 ? ensure_split(c, pc * (c->nt - 1), Smax) : GPF_OK;
}

// One k_step launch of a factorisation: block column J of particle group g (particles
// [p0, p0+gc) of the chunk, on that group's stream), its kernel variant, grid, pieces per split
// tile, and where its split-K partial slots and arrival counters start (element offsets into
// d_part / d_cnt). run_factor launches exactly this list; gpf_plan_check verifies it on the host.
struct StepLaunch {
  int J, g, p0, gc, split, S, S2, grp, ed;  // S: pieces per split tile (SPLIT_ALL: chunks per piece); S2: partial
                                            // slots per tile; ed: the launch starts with gc diagonal workgroups
  int defer, sy;                        // deferred diagonal update; sy: gc SYRK workgroups follow
  int ro;  // reordered dispatch (gpf::step_decode ro): light U tiles, diagonal, other tiles, SYRK workgroups
  int la;  // look-ahead: bit 0: gc LA workgroups follow (gpf::la_item); bit 1: the critical tiles seed from launch J-1's
  int pair;  // paired block columns: 1 lead launch (gpf::pair_decode), 2 follow launch (its tiles seed from the lead's partials)
  unsigned grid;
  size_t part_off, cnt_off;
};

static unsigned one_per_cu_lds(const StepLaunch& l) {
  const int on = getenv("GPF_STEP_1PERCU") ? atoi(getenv("GPF_STEP_1PERCU")) : 0;
  if (!on || !l.ed || l.split != gpf::SPLIT_NONE) return 0;
  return (unsigned)(82 * 1024 - gpf::STEP_LDS * 8);  // > 80 KiB in all: one per CU
}

static void step_plan(int pc, int nt, int S, int Smax, std::vector<StepLaunch>& out) {
  out.clear();
  const int ng = num_groups(pc, nt);
  const bool ed = early_diag(pc, nt);
  // block columns interleaved across groups so every stream has work queued early
  for (int J = 0; nt > 1 && J < nt; ++J) {
    for (int g = 0; g < ng; ++g) {
      StepLaunch l{};
      l.J = J;
      l.g = g;
      l.p0 = (int)((long long)pc * g / ng);
      l.gc = (int)((long long)pc * (g + 1) / ng) - l.p0;
      l.grp = step_group(l.gc);
      l.S = S > 1 ? split_all_target(l.gc, nt, J) : 1;
      l.S2 = S > 1 ? Smax : 1;
      l.split = S > 1 ? gpf::SPLIT_ALL : gpf::SPLIT_NONE;
      l.ed = ed ? 1 : 0;
      l.defer = (S == 1 && defer_syrk()) ? 1 : 0;  // the all-tile split keeps the per-tile look-ahead
      l.sy = (l.defer && J >= 1 && J <= nt - 2) ? 1 : 0;
      // look-ahead: launch J-1 of this group must have run unsplit too (its LA workgroups)
      const bool la_ok = look_ahead(pc, nt) && l.ed && l.split == gpf::SPLIT_NONE;
      const bool prev_none = J >= 1 && S == 1;
      const bool next_none = S == 1;
      l.la = ((la_ok && next_none && J >= 1 && J <= nt - 3) ? 1 : 0) | ((la_ok && prev_none && J >= 2 && J <= nt - 2) ? 2 : 0);
      // reordered dispatch: only where the first 3 gc workgroups (the light U tiles, which wait for
      // the diagonal workgroups behind them, and the SYRK workgroups) fit the chip's CUs at once
      // and one group (a concurrent group's launch could hold the slots the waiters need)
      l.ro = (reorder_on() && ng == 1 && l.ed && l.sy && l.split == gpf::SPLIT_NONE && l.grp == 0 && J >= 1 &&
              3 * l.gc <= 256) ? 1 : 0;
      // paired block columns: leads at odd J with a block column behind them, each followed by J+1
      const bool pairs = pair_on() && !l.ed && S == 1 && l.defer && l.grp == 0 && l.gc % 8 == 0 && nt >= 4;
      l.pair = pairs && (J & 1) && J + 1 <= nt - 1 ? 1 : (pairs && J >= 2 && !(J & 1) ? 2 : 0);
      if (l.pair == 2) l.sy = 0;  // (the lead's partial SYRK and the critical tile reduce the diagonal block)
      int nall = 0;
      for (int w = 0; S > 1 && w < nt - 1; ++w) nall += gpf::split_all_pieces(J, w, nt, l.S);
      l.grid = (S > 1 ? l.gc * nall : l.gc * (nt - 1)) + (l.ed ? l.gc : 0) + (l.sy ? l.gc : 0) +
               ((l.la & 1) && !l.sy ? l.gc : 0);  // (with SYRK workgroups the look-ahead rides on them)
      if (l.pair == 1) l.grid = (unsigned)(l.gc * gpf::pair_grid_per_particle(J, nt));
      // all-tile look-ahead (early-diagonal launches): bit 0 this launch produces pieces for J+1, bit 1
      // its tiles and SYRK workgroup consume launch J-1's
      const int j0 = lall_from(nt);
      if (lall_on() && l.ed && S == 1 && l.defer && nt >= 4 && nt <= LALL_NT_MAX && J >= j0) {
        // launches J >= j0 produce pieces for J+1, launches J > j0 consume them (and run no
        // critical-tile look-ahead: the pieces carry the next critical tile too); launch j0 may still
        // seed its critical tile from launch j0-1's look-ahead
        l.pair = (gpf::lall_items(J, nt) > 0 ? 1 : 0) | (J >= 2 && J > j0 ? 2 : 0);
        if ((l.pair & 1) && lall_first()) l.pair |= 4;
        l.la = J > j0 ? 0 : (l.la & 2);
        l.ro = 0;
        l.grid = (unsigned)(l.gc * (nt - 1) + l.gc + (l.sy ? l.gc : 0) + l.gc * gpf::lall_total(J, nt, lall_pb()));
      }
      // one set of partial slots per group: groups run concurrently
      l.part_off = (size_t)l.p0 * (nt - 1) * Smax * T * T;
      l.cnt_off = (size_t)l.p0 * (nt - 1) * gpf::split_cnt_stride(nt);
      out.push_back(l);
    }
  }
}

// Factorise `pc` particles whose length scales are already in d_ls, in particle
// groups on their own streams: per group the K build (the 128-wide diagonal blocks), then one
// k_step per 128-wide block column. With the fused diagonal factor (early_diag false) k_diag
// factors block 0 first and each launch J factors block J+1 at the end of its critical tile;
// with the early diagonal factor launch J itself starts with the factor of block J. Joins back
// into c->stream.
static int run_factor(gpf_ctx* c, int pc) {
  const int nt = c->nt, Np = (int)c->Npad, N = (int)c->N;
  const double Tf = (double)T, t3 = Tf * Tf * Tf;
  const int nb = Np / BT;
  const int ntri = nb * (nb + 1) / 2;
  const size_t ld = (size_t)Np;
  const int ng = num_groups(pc, nt);
  const bool persist = persist_on(pc, nt);
  // algorithmic flops of block-column launch J per particle, potrf + trtri (2/3 N^3) formulation:
  //   L tile: depth-128J GEMM 2 T^3 J + triangular multiply T^3 + look-ahead syrk share T^3
  //   U tile: depth-128(J-K) GEMM with a triangular factor 2 T^3 (J-K) - T^3 + triangular multiply T^3
  //   diagonal block: 2/3 T^3 (block J+1 fused at the end of launch J, or block J early in it)
  const bool ed = !persist && early_diag(pc, nt);
  const int spins = wait_spins();
  auto step_flops = [&](int J) {
    double fl = 0.0;
    for (int w = 0; w < nt - 1; ++w) {
      if (w < nt - 1 - J) fl += 2.0 * t3 * J + 2.0 * t3;
      else fl += 2.0 * t3 * (J - (w - (nt - 1 - J)));
    }
    if (ed || J + 1 < nt) fl += (2.0 / 3.0) * t3;
    return fl;
  };
  // paired block columns: the lead launch J also runs block column J+1's GEMMs over the columns < J
  // (L tiles I >= J+2: depth 128J; U tiles K < J: depth 128(J-K), first block triangular), which the
  // follow launch then does not
  auto pla_flops = [&](int J) {
    double fl = 0.0;
    for (int w = 1; w < nt - 1; ++w) {
      if (w < nt - 1 - J) fl += 2.0 * t3 * J;
      else fl += 2.0 * t3 * (J - (w - (nt - 1 - J))) - t3;
    }
    return fl;
  };
  // Split-K plan first: a (re)allocation of the arrival counters queues their zeroing memset on
  // c->stream, which must precede the fork event the group streams wait on (with ng > 1 the
  // k_step launches run on the sub-streams, and an unordered memset could land after a piece
  // took its ticket, leaving a tile unfinished).
  int S = 1, Smax = 1;
  if (int rc = split_plan(c, pc, S, Smax)) return rc;
  // the split-K tickets and ready flags start at zero in every split factorisation: the
  // finishing pieces re-zero what they used, but a hand-off that timed out (info bit 2) leaves its
  // pair's ticket and flag set, and the next tree would elect the wrong finisher;
  // ~20 KB at N=4096 for one particle, on c->stream ahead of the fork
  if (Smax > 1)
    GPF_HIP(c, hipMemsetAsync(c->d_cnt, 0, (size_t)pc * (nt - 1) * gpf::split_cnt_stride(nt) * 4, c->stream));
  hipEvent_t wa = nullptr, wb = nullptr;
  if (c->prof) {
    wa = take_event(c);
    wb = take_event(c);
    if (wa && wb) hipEventRecord(wa, c->stream);
  }
  if (ng > 1) {
    GPF_HIP(c, hipEventRecord(c->fork, c->stream));
    for (int g = 0; g < ng; ++g) GPF_HIP(c, hipStreamWaitEvent(c->sub[g], c->fork, 0));
  }
  double total = 0.0;
  for (int g = 0; g < ng; ++g) {
    const int p0 = (int)((long long)pc * g / ng), gc = (int)((long long)pc * (g + 1) / ng) - p0;
    hipStream_t st = (ng > 1) ? c->sub[g] : c->stream;
    double* Lg = c->d_L + (size_t)p0 * ld * ld;
    double* Ug = c->d_U + (size_t)p0 * ld * ld;
    double* yg = c->d_yb + (size_t)p0 * ld;
    double* s2g = c->d_s2p + (size_t)p0 * nt * ld;
    double* szg = c->d_szp + (size_t)p0 * nt * ld;
    int* ig = c->d_info + p0;
    const double* lsg = c->d_ls + (size_t)p0 * c->d;
    // only the diagonal blocks are built here; k_step computes the other tiles
    const int nbuild = nt > 1 ? 3 * nt : ntri;
    int rc = launch_on(c, st, PC_BUILD, 8.0 * nbuild * BT * BT * (double)gc, [&] {
      hipLaunchKernelGGL(gpf::k_build_cov, dim3(nbuild, gc), dim3(NTHR), 0, st, N, Np, c->d, c->d_x, c->d_y, c->d_e,
                         lsg, Lg, yg, ig, (int)(nbuild != ntri), c->d_flag + p0, c->d_cflag + p0,
                         persist ? c->d_pst : nullptr, (long long)c->cap * nt, nt);
    });
    if (rc) return rc;
    if (ed) continue;  // block 0 is factored by launch 0's diagonal workgroups
    // potrf + trtri of the first 128 block: 2/3 T^3 (later blocks are fused into k_step)
    rc = launch_on(c, st, PC_DIAG, (2.0 / 3.0) * t3 * gc, [&] {
      hipLaunchKernelGGL(gpf::k_diag, dim3(gc), dim3(gpf::DNTH), 0, st, 0, nt, N, Np, Lg, Ug, yg, s2g, szg, ig,
                         c->d_flag + p0);
    });
    if (rc) return rc;
    total += (2.0 / 3.0) * t3 * gc;
  }
  if (persist) {
    // one persistent launch: every block column of every particle (gpf_persist.hip)
    double fl = 0.0;
    for (int J = 0; J < nt; ++J) fl += step_flops(J);
    gpf::PItem a{nt, Np, N, c->d, spins, c->d_L, c->d_U, c->d_yb, c->d_s2p, c->d_szp, c->d_info, c->d_x, c->d_ls};
    const size_t ps = (size_t)c->cap * nt;
    gpf::PState ps_{c->d_pst, c->d_pst + ps, c->d_pst + 2 * ps, reinterpret_cast<unsigned*>(c->d_pst + 3 * ps),
                    c->d_pst + 3 * ps + gpf::PQ_MAX};
    const int rc = launch_on(c, c->stream, PC_PANEL, fl * pc, [&] {
      hipLaunchKernelGGL(gpf::k_factor, dim3((unsigned)gpf::p_total_items(pc, nt)), dim3(gpf::STEP_NTH), 0, c->stream, a,
                         ps_, pc, c->prof ? c->d_clk : nullptr);
    });
    if (rc) return rc;
    total += fl * pc;
    if (c->prof && wa && wb) {
      hipEventRecord(wb, c->stream);
      c->pend.push_back({wa, wb, PC_FACTOR, total});
    }
    return GPF_OK;
  }
  // block-column launches (split-K for launches with few tiles, planned above)
  std::vector<StepLaunch> plan;
  step_plan(pc, nt, S, Smax, plan);
  bool any_la = false, any_pair = false;
  for (const StepLaunch& l : plan) {
    any_la = any_la || l.la != 0;
    any_pair = any_pair || (!l.ed && l.pair != 0);
  }
  const size_t pb_bytes = (size_t)pc * (nt - 1) * T * T * 8;
  if (any_pair && pb_bytes > c->pb_cap) {  // (nt >= 4: never under a graph capture)
    clear_graphs(c);
    hipFree(c->d_pb);
    c->d_pb = nullptr;
    c->pb_cap = 0;
    GPF_HIP(c, hipMalloc(&c->d_pb, pb_bytes));
    c->pb_cap = pb_bytes;
  }
  const size_t ps_bytes = (size_t)pc * (nt - 1) * gpf::PAIR_HMAX * 4;
  if (any_pair && ps_bytes > c->pstart_cap) {
    hipFree(c->d_pstart);
    c->d_pstart = nullptr;
    c->pstart_cap = 0;
    GPF_HIP(c, hipMalloc(&c->d_pstart, ps_bytes));
    GPF_HIP(c, hipMemset(c->d_pstart, 0, ps_bytes));  // (tags start at 1)
    c->pstart_cap = ps_bytes;
  }
  bool any_lall = false;
  for (const StepLaunch& l : plan) any_lall = any_lall || (l.ed && l.pair != 0);
  const int smax = lall_smax(nt);
  const size_t lb_bytes = (size_t)2 * pc * smax * T * T * 8;
  if (any_lall && lb_bytes > c->lb_cap) {
    clear_graphs(c);
    hipFree(c->d_lb);
    c->d_lb = nullptr;
    c->lb_cap = 0;
    GPF_HIP(c, hipMalloc(&c->d_lb, lb_bytes));
    c->lb_cap = lb_bytes;
  }
  const int seq = ++c->fact_seq & 0x7fffff;
  const bool psync = getenv("GPF_PAIR_SYNC") == nullptr || atoi(getenv("GPF_PAIR_SYNC")) != 0;
  if (any_la && 2 * (size_t)pc * T * T * 8 > c->la_cap) {  // (never under a graph capture: nt >= 4 only)
    clear_graphs(c);
    hipFree(c->d_la);
    c->d_la = nullptr;
    c->la_cap = 0;
    GPF_HIP(c, hipMalloc(&c->d_la, 2 * (size_t)pc * T * T * 8));  // two slots per particle (gpf::la_slot)
    c->la_cap = 2 * (size_t)pc * T * T * 8;
  }
  // test hook: the critical tiles that seed from the look-ahead wait ~0.3 ms first (gpf::step_item)
  const int la_delay = (getenv("GPF_LA_DELAY_TEST") && atoi(getenv("GPF_LA_DELAY_TEST")) != 0) ? 4 : 0;
  for (const StepLaunch& l : plan) {
    // (paired columns: lead 1, follow 2; look-ahead pieces: bit 0 produces for J+1, bit 1 consumes J-1's —
    // either way the GEMMs over the columns < J of block column J+1's tiles move one launch earlier)
    const double fl = step_flops(l.J) + ((l.pair & 1) ? pla_flops(l.J) : 0.0) - ((l.pair & 2) ? pla_flops(l.J - 1) : 0.0);
    const int p0 = l.p0, gc = l.gc;
    hipStream_t st = (ng > 1) ? c->sub[l.g] : c->stream;
    // (every split launch gets its buffers: under SPLIT_ALL, l.S is chunks per piece, not a piece count)
    double* partg = l.split != gpf::SPLIT_NONE ? c->d_part + l.part_off : nullptr;
    unsigned* cntg = l.split != gpf::SPLIT_NONE ? c->d_cnt + l.cnt_off : nullptr;
    if (l.split == gpf::SPLIT_ALL && !ed) return bad_arg(c, "internal: all-tile split without the early diagonal factor");
    const auto kern = l.split == gpf::SPLIT_ALL ? gpf::k_step<gpf::SPLIT_ALL, 1>
                                                : (ed ? gpf::k_step<gpf::SPLIT_NONE, 1> : gpf::k_step<gpf::SPLIT_NONE, 0>);
    const int rc = launch_on(c, st, PC_PANEL, fl * gc, [&] {
      hipLaunchKernelGGL(kern, dim3(l.grid), dim3(gpf::STEP_NTH), one_per_cu_lds(l), st, l.J, nt, Np, c->d_L + (size_t)p0 * ld * ld,
                         c->d_U + (size_t)p0 * ld * ld, c->d_yb + (size_t)p0 * ld, c->d_s2p + (size_t)p0 * nt * ld,
                         c->d_szp + (size_t)p0 * nt * ld, c->d_info + p0, gc, l.grp, N, c->d_x,
                         c->d_ls + (size_t)p0 * c->d, c->d, l.S, l.S2, partg, cntg, c->d_flag + p0, l.ed,
                         c->d_cflag + p0, l.defer, l.sy, spins,
                         l.la | ((l.la & 2) ? la_delay : 0) | (l.ro ? 32 : 0),
                         l.la ? c->d_la + 2 * (size_t)p0 * T * T : nullptr, l.pair,
                         l.pair ? (l.ed ? c->d_lb + (size_t)2 * p0 * smax * T * T : c->d_pb + gpf::pair_slot(p0, 0, nt))
                                : nullptr,
                         (!l.ed && l.pair == 1 && psync) ? c->d_pstart + (size_t)p0 * (nt - 1) * gpf::PAIR_HMAX : nullptr,
                         l.ed ? gpf::lall_tag(gc, lall_pb(), smax) : (seq << 8) | l.J, c->prof ? c->d_clk : nullptr);
    });
    if (rc) return rc;
    total += fl * gc;
  }
  if (ng > 1) {
    for (int g = 0; g < ng; ++g) {
      GPF_HIP(c, hipEventRecord(c->join[g], c->sub[g]));
      GPF_HIP(c, hipStreamWaitEvent(c->stream, c->join[g], 0));
    }
  }
  if (c->prof && wa && wb) {
    hipEventRecord(wb, c->stream);
    c->pend.push_back({wa, wb, PC_FACTOR, total});
  }
  return GPF_OK;
}

// ---- convex-hull grid fill helpers (convex_hull.py:122-155,203-224) ----
namespace {
struct DevBuf {  // owning device allocation, stream-ordered (no device-wide sync on free)
  void* p = nullptr;
  hipStream_t st = nullptr;
  hipError_t alloc(size_t bytes, hipStream_t s) {
    st = s;
    return hipMallocAsync(&p, bytes, s);
  }
  ~DevBuf() { if (p) hipFreeAsync(p, st); }
  template <typename V> V* as() { return static_cast<V*>(p); }
};
inline unsigned blocks_for(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + NTHR - 1) / NTHR); }
}  // namespace

// Sort rows (n x d, device) lexicographically by columns order[0], order[1], ... (stable LSD
// sequence of radix sorts) and drop repeated rows; rows/n are replaced by the result.
static int hull_sort_unique(gpf_ctx* c, DevBuf& rows, int64_t& n, int d, const int* order) {
  hipStream_t st = c->stream;
  DevBuf perm, perm2, key, key2, flag, pos, temp, out;
  GPF_HIP(c, perm.alloc(std::max<int64_t>(n, 1) * 8, st));
  GPF_HIP(c, perm2.alloc(std::max<int64_t>(n, 1) * 8, st));
  GPF_HIP(c, key.alloc(std::max<int64_t>(n, 1) * 8, st));
  GPF_HIP(c, key2.alloc(std::max<int64_t>(n, 1) * 8, st));
  hipLaunchKernelGGL(gpf::k_hull_iota, dim3(blocks_for(n)), dim3(NTHR), 0, st, perm.as<int64_t>(), n);
  size_t tb = 0, tb2 = 0;
  GPF_HIP(c, hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key.as<uint64_t>(), key2.as<uint64_t>(),
                                                perm.as<int64_t>(), perm2.as<int64_t>(), n, 0, 64, st));
  GPF_HIP(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, perm.as<int64_t>(), perm2.as<int64_t>(), n, st));
  GPF_HIP(c, temp.alloc(std::max<size_t>(std::max(tb, tb2), 16), st));
  for (int q = d - 1; q >= 0; --q) {
    hipLaunchKernelGGL(gpf::k_hull_key, dim3(blocks_for(n)), dim3(NTHR), 0, st, rows.as<double>(),
                       perm.as<int64_t>(), n, d, order[q], key.as<uint64_t>());
    GPF_HIP(c, hipcub::DeviceRadixSort::SortPairs(temp.p, tb, key.as<uint64_t>(), key2.as<uint64_t>(),
                                                  perm.as<int64_t>(), perm2.as<int64_t>(), n, 0, 64, st));
    std::swap(perm.p, perm2.p);
  }
  GPF_HIP(c, flag.alloc(std::max<int64_t>(n, 1) * 8, st));
  GPF_HIP(c, pos.alloc(std::max<int64_t>(n, 1) * 8, st));
  hipLaunchKernelGGL(gpf::k_hull_flag, dim3(blocks_for(n)), dim3(NTHR), 0, st, rows.as<double>(), perm.as<int64_t>(),
                     n, d, flag.as<int64_t>());
  GPF_HIP(c, hipcub::DeviceScan::ExclusiveSum(temp.p, tb2, flag.as<int64_t>(), pos.as<int64_t>(), n, st));
  int64_t last[2] = {0, 0};
  GPF_HIP(c, hipMemcpyAsync(&last[0], pos.as<int64_t>() + (n - 1), 8, hipMemcpyDeviceToHost, st));
  GPF_HIP(c, hipMemcpyAsync(&last[1], flag.as<int64_t>() + (n - 1), 8, hipMemcpyDeviceToHost, st));
  GPF_HIP(c, hipStreamSynchronize(st));
  const int64_t m = last[0] + last[1];
  GPF_HIP(c, out.alloc(std::max<int64_t>(m, 1) * d * 8, st));
  hipLaunchKernelGGL(gpf::k_hull_compact, dim3(blocks_for(n)), dim3(NTHR), 0, st, rows.as<double>(),
                     perm.as<int64_t>(), flag.as<int64_t>(), pos.as<int64_t>(), n, d, out.as<double>());
  GPF_HIP(c, hipGetLastError());
  GPF_HIP(c, hipStreamSynchronize(st));
  std::swap(rows.p, out.p);
  n = m;
  return GPF_OK;
}

extern "C" {

#ifndef GPF_BUILD_INFO
#define GPF_BUILD_INFO "unknown"
#endif
int gpf_version(void) { return GPF_ABI_VERSION; }
const char* gpf_build_info(void) { return GPF_BUILD_INFO; }
int gpf_tile(void) { return T; }

int gpf_open(int device, gpf_ctx** out) {
  if (!out) return GPF_BAD_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return GPF_HIP_ERROR;
  if (device < 0 || device >= n) return GPF_BAD_ARG;
  if (hipSetDevice(device) != hipSuccess) return GPF_HIP_ERROR;
  gpf_ctx* c = new gpf_ctx();
  c->device = device;
  if (hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c->ncu <= 0) c->ncu = 256;
  bool ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreateWithFlags(&c->fork, hipEventDisableTiming) == hipSuccess;
  for (int g = 0; ok && g < MAX_GROUPS; ++g)
    ok = hipStreamCreateWithFlags(&c->sub[g], hipStreamNonBlocking) == hipSuccess &&
         hipEventCreateWithFlags(&c->join[g], hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    gpf_close(c);
    return GPF_HIP_ERROR;
  }
  *out = c;
  return GPF_OK;
}

void gpf_close(gpf_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  harvest(c);
  free_work(c);
  hipFree(c->d_x); hipFree(c->d_y); hipFree(c->d_e);
  hipFree(c->d_clk);
  hipFree(c->d_sig); hipFree(c->d_exp); hipFree(c->d_lo); hipFree(c->d_hi);
  hipFree(c->km_x); hipFree(c->km_c); hipFree(c->km_dist); hipFree(c->km_sums); hipFree(c->km_cnt); hipFree(c->km_lab);
  for (auto e : c->pool) hipEventDestroy(e);
  for (int g = 0; g < MAX_GROUPS; ++g) {
    if (c->sub[g]) hipStreamDestroy(c->sub[g]);
    if (c->join[g]) hipEventDestroy(c->join[g]);
  }
  if (c->fork) hipEventDestroy(c->fork);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

const char* gpf_last_error(gpf_ctx* c) { return c ? c->err.c_str() : "null context"; }

int gpf_set_data(gpf_ctx* c, const double* x, const double* y, const double* e, int64_t N, int d) {
  if (!c) return GPF_BAD_ARG;
  if (N <= 0 || d <= 0 || !x || !y || !e) return bad_arg(c, "gpf_set_data: empty or null input");
  if (d > gpf::DMAX) return bad_arg(c, "gpf_set_data: d exceeds DMAX (32)");
  if (N > (int64_t)1 << 20) return bad_arg(c, "gpf_set_data: N too large");
  hipSetDevice(c->device);
  GPF_HIP(c, hipStreamSynchronize(c->stream));
  free_work(c);
  hipFree(c->d_x); hipFree(c->d_y); hipFree(c->d_e);
  c->d_x = c->d_y = c->d_e = nullptr;
  c->N = N;
  c->d = d;
  c->nt = (int)((N + T - 1) / T);
  c->Npad = (int64_t)c->nt * T;
  GPF_HIP(c, hipMalloc(&c->d_x, (size_t)N * d * 8));
  GPF_HIP(c, hipMalloc(&c->d_y, (size_t)N * 8));
  GPF_HIP(c, hipMalloc(&c->d_e, (size_t)N * 8));
  GPF_HIP(c, hipMemcpy(c->d_x, x, (size_t)N * d * 8, hipMemcpyHostToDevice));
  GPF_HIP(c, hipMemcpy(c->d_y, y, (size_t)N * 8, hipMemcpyHostToDevice));
  GPF_HIP(c, hipMemcpy(c->d_e, e, (size_t)N * 8, hipMemcpyHostToDevice));
  c->h_y.assign(y, y + N);
  return GPF_OK;
}

int gpf_set_grid(gpf_ctx* c, const double* sig, const double* expct, int K, const double* lo, const double* hi) {
  if (!c) return GPF_BAD_ARG;
  if (c->d <= 0) return bad_arg(c, "gpf_set_grid: call gpf_set_data first");
  if (K < 2 || K > gpf::KGRID_MAX || !sig || !expct || !lo || !hi) return bad_arg(c, "gpf_set_grid: bad grid");
  hipSetDevice(c->device);
  GPF_HIP(c, hipStreamSynchronize(c->stream));
  if (K != c->K) {
    free_work(c);  // histogram size depends on K
    hipFree(c->d_sig); hipFree(c->d_exp);
    c->d_sig = c->d_exp = nullptr;
    GPF_HIP(c, hipMalloc(&c->d_sig, (size_t)K * 8));
    GPF_HIP(c, hipMalloc(&c->d_exp, (size_t)K * 8));
  }
  if (!c->d_lo) {
    GPF_HIP(c, hipMalloc(&c->d_lo, gpf::DMAX * 8));
    GPF_HIP(c, hipMalloc(&c->d_hi, gpf::DMAX * 8));
  }
  c->K = K;
  GPF_HIP(c, hipMemcpy(c->d_sig, sig, (size_t)K * 8, hipMemcpyHostToDevice));
  GPF_HIP(c, hipMemcpy(c->d_exp, expct, (size_t)K * 8, hipMemcpyHostToDevice));
  GPF_HIP(c, hipMemcpy(c->d_lo, lo, (size_t)c->d * 8, hipMemcpyHostToDevice));
  GPF_HIP(c, hipMemcpy(c->d_hi, hi, (size_t)c->d * 8, hipMemcpyHostToDevice));
  c->h_lo.assign(lo, lo + c->d);
  c->h_hi.assign(hi, hi + c->d);
  return GPF_OK;
}

int gpf_eval_batch(gpf_ctx* c, const double* ls, int P, double* loss, double* mu, double* sd, int* bad_idx) {
  if (!c) return GPF_BAD_ARG;
  if (bad_idx) *bad_idx = -1;
  if (P < 0 || (P > 0 && (!ls || !loss))) return bad_arg(c, "gpf_eval_batch: bad arguments");
  if (c->N <= 0 || c->K <= 0) return bad_arg(c, "gpf_eval_batch: call gpf_set_data and gpf_set_grid first");
  hipSetDevice(c->device);
  const int d = c->d;
  const int64_t N = c->N, Np = c->Npad;
  // sentinel particles (find_len_scales.py:156-157) never reach the GPU
  std::vector<int> act;
  act.reserve(P);
  for (int p = 0; p < P; ++p) {
    bool out = false;
    for (int k = 0; k < d; ++k) {
      const double v = ls[(size_t)p * d + k];
      if (v <= c->h_lo[k] || v >= c->h_hi[k]) out = true;
    }
    if (out) {
      loss[p] = 1e13;
      if (mu) for (int64_t i = 0; i < N; ++i) mu[(size_t)p * N + i] = NAN;
      if (sd) for (int64_t i = 0; i < N; ++i) sd[(size_t)p * N + i] = NAN;
    } else {
      act.push_back(p);
    }
  }
  if (act.empty()) return GPF_OK;
  // Enqueue one chunk of pc particles whose length scales are staged in c->h_ls.
  auto enqueue = [&](int pc) -> int {
    GPF_HIP(c, hipMemcpyAsync(c->d_ls, c->h_ls, (size_t)pc * d * 8, hipMemcpyHostToDevice, c->stream));
    int r = run_factor(c, pc);
    if (r) return r;
    r = launch(c, PC_LOSS, 0.0, [&] {
      hipLaunchKernelGGL(gpf::k_points, dim3((unsigned)((N + NTHR - 1) / NTHR), pc), dim3(NTHR), 0, c->stream,
                         (int)N, (int)Np, c->nt, c->K, c->d_y, c->d_e, c->d_sig, c->d_s2p, c->d_szp, c->d_mu,
                         c->d_sd, c->d_hist);
      hipLaunchKernelGGL(gpf::k_score, dim3(pc), dim3(NTHR), 0, c->stream, (int)N, c->K, d, c->d_sig, c->d_exp,
                         c->d_hist, c->d_ls, c->d_lo, c->d_hi, c->d_loss);
    });
    if (r) return r;
    GPF_HIP(c, hipMemcpyAsync(c->h_loss, c->d_loss, (size_t)pc * 8, hipMemcpyDeviceToHost, c->stream));
    GPF_HIP(c, hipMemcpyAsync(c->h_info, c->d_info, (size_t)pc * 4, hipMemcpyDeviceToHost, c->stream));
    return GPF_OK;
  };
  // Small problems are launch-latency bound: the whole batch (copies + ~5 kernels) is
  // captured once per batch size as a HIP graph and replayed. The batch is padded to all P
  // slots (spare slots repeat an active particle) so one graph serves every PSO iteration.
  // (Replaying graphs of the live particles up to N = 1920 measured no gain at N = 1024: the
  // ~10 us between dependent k_step launches is not launch overhead; profiles/r1/split_crit_ab.txt.)
  const bool graph = !c->prof && !mu && !sd && c->nt <= GRAPH_NT_MAX && getenv("GPF_NO_GRAPH") == nullptr;
  if (graph) {
    int rc = ensure_work(c, P);
    if (rc) return rc;
    if (c->cap >= P) {
      for (int q = 0; q < P; ++q) {
        const int src = act[q < (int)act.size() ? q : 0];
        for (int k = 0; k < d; ++k) c->h_ls[(size_t)q * d + k] = ls[(size_t)src * d + k];
      }
      hipGraphExec_t ge = nullptr;
      for (auto& g : c->graphs)
        if (g.first == P) ge = g.second;
      if (!ge) {
        GPF_HIP(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
        const int rq = enqueue(P);
        hipGraph_t gr = nullptr;
        const hipError_t ec = hipStreamEndCapture(c->stream, &gr);
        if (rq) {
          if (gr) hipGraphDestroy(gr);
          return rq;
        }
        GPF_HIP(c, ec);
        const hipError_t ei = hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
        hipGraphDestroy(gr);
        GPF_HIP(c, ei);
        if (c->graphs.size() >= 8) {  // bounded cache: drop the oldest batch size
          hipGraphExecDestroy(c->graphs.front().second);
          c->graphs.erase(c->graphs.begin());
        }
        c->graphs.push_back({P, ge});
      }
      GPF_HIP(c, hipGraphLaunch(ge, c->stream));
      GPF_HIP(c, hipStreamSynchronize(c->stream));
      c->evals += (double)act.size();
      for (size_t q = 0; q < act.size(); ++q) {
        if (c->h_info[q] & 2) {
          c->err = "k_step: diagonal-block hand-off timed out";
          return GPF_HIP_ERROR;
        }
        if (c->h_info[q] != 0) {
          if (bad_idx) *bad_idx = act[q];
          c->err = "Matrix is not positive definite";
          return GPF_NOT_PD;
        }
        loss[act[q]] = c->h_loss[q];
      }
      return GPF_OK;
    }
  }
  int rc = ensure_work(c, (int)act.size());
  if (rc) return rc;
  const int cap = c->cap;
  std::vector<double> hmu, hsd;
  if (mu) hmu.resize((size_t)cap * Np);
  if (sd) hsd.resize((size_t)cap * Np);
  for (size_t s = 0; s < act.size(); s += cap) {
    const int pc = (int)std::min<size_t>(cap, act.size() - s);
    for (int q = 0; q < pc; ++q)
      for (int k = 0; k < d; ++k) c->h_ls[(size_t)q * d + k] = ls[(size_t)act[s + q] * d + k];
    rc = enqueue(pc);
    if (rc) return rc;
    if (mu) GPF_HIP(c, hipMemcpyAsync(hmu.data(), c->d_mu, (size_t)pc * Np * 8, hipMemcpyDeviceToHost, c->stream));
    if (sd) GPF_HIP(c, hipMemcpyAsync(hsd.data(), c->d_sd, (size_t)pc * Np * 8, hipMemcpyDeviceToHost, c->stream));
    GPF_HIP(c, hipStreamSynchronize(c->stream));
    if (c->prof) harvest(c);
    c->evals += pc;
    for (int q = 0; q < pc; ++q) {
      const int p = act[s + q];
      if (c->h_info[q] & 2) {
        c->err = "k_step: diagonal-block hand-off timed out";
        return GPF_HIP_ERROR;
      }
      if (c->h_info[q] != 0) {
        if (bad_idx) *bad_idx = p;
        c->err = "Matrix is not positive definite";
        return GPF_NOT_PD;
      }
      loss[p] = c->h_loss[q];
      if (mu) std::memcpy(mu + (size_t)p * N, hmu.data() + (size_t)q * Np, (size_t)N * 8);
      if (sd) std::memcpy(sd + (size_t)p * N, hsd.data() + (size_t)q * Np, (size_t)N * 8);
    }
  }
  return GPF_OK;
}

// Factorise one particle (slot 0 of the workspace) without waiting: the factor's status word is
// copied to the pinned c->h_info[0] behind it on c->stream, and the caller checks it (factor_status)
// after its next synchronisation — gpf_predict queues the query kernels right behind the
// factorisation instead of idling the GPU for a host round trip. ls == nullptr: the length scales
// are already in d_ls (queued on c->stream by the caller). alpha_out (nullable): alpha = K^-1 y
// into the mu slot of particle 0 (gpf_predict forms its mean from V^T z and does not need it).
static int factor_single_async(gpf_ctx* c, const double* ls, double** alpha_out) {
  int rc = ensure_work(c, 1);
  if (rc) return rc;
  if (ls) {
    std::memcpy(c->h_ls, ls, (size_t)c->d * 8);
    GPF_HIP(c, hipMemcpyAsync(c->d_ls, c->h_ls, (size_t)c->d * 8, hipMemcpyHostToDevice, c->stream));
  }
  GPF_HIP(c, hipMemsetAsync(c->d_info, 0, 4, c->stream));
  rc = run_factor(c, 1);
  if (rc) return rc;
  if (alpha_out) {
    rc = launch(c, PC_LOSS, 0.0, [&] {
      hipLaunchKernelGGL(gpf::k_alpha, dim3((unsigned)((c->N + NTHR - 1) / NTHR)), dim3(NTHR), 0, c->stream,
                         (int)c->N, (int)c->Npad, c->nt, c->d_szp, c->d_mu);
    });
    if (rc) return rc;
    *alpha_out = c->d_mu;
  }
  GPF_HIP(c, hipMemcpyAsync(c->h_info, c->d_info, 4, hipMemcpyDeviceToHost, c->stream));
  return GPF_OK;
}

// The status of the last factor_single_async (valid once c->stream has been synchronised).
static int factor_status(gpf_ctx* c) {
  const int info = c->h_info[0];
  if (info & 2) {
    c->err = "k_step: diagonal-block hand-off timed out";
    return GPF_HIP_ERROR;
  }
  if (info != 0) {
    c->err = "Matrix is not positive definite";
    return GPF_NOT_PD;
  }
  return GPF_OK;
}

static int factor_single(gpf_ctx* c, const double* ls, double** alpha_out) {
  int rc = factor_single_async(c, ls, alpha_out);
  if (rc) return rc;
  GPF_HIP(c, hipStreamSynchronize(c->stream));
  rc = factor_status(c);
  if (rc) *alpha_out = nullptr;
  return rc;
}

int gpf_predict(gpf_ctx* c, const double* ls, const double* xfit, int64_t M, int64_t batch, double* mu,
                double* sd) {
  if (!c) return GPF_BAD_ARG;
  if (c->N <= 0) return bad_arg(c, "gpf_predict: call gpf_set_data first");
  if (M < 0 || (M > 0 && (!xfit || !mu || !sd)) || !ls) return bad_arg(c, "gpf_predict: bad arguments");
  if (M == 0) return GPF_OK;
  hipSetDevice(c->device);
  if (c->K <= 0) {  // predict does not need the objective grid; size the histogram minimally
    c->K = 2;
  }
  // Query chunk: as large as memory allows (the reference's batch_size only bounds its
  // own host memory, GP_func.py:28-30; results do not depend on it). Sized before the
  // factorisation is queued, so that a (re)allocation never waits for it; free memory is only
  // queried when the kept buffers are too small.
  // the factorisation workspace first: a (re)allocation there frees the query buffers too
  if (int rw = ensure_work(c, 1)) return rw;
  const int64_t Np = c->Npad;
  int64_t chunk = std::min<int64_t>(std::max<int64_t>(std::max<int64_t>(batch, 1), 16384), M);
  int64_t Cp = ((chunk + T - 1) / T) * T;
  const bool fits = c->p_cols >= Cp && c->p_np == Np && c->p_d == c->d && c->p_nt == c->nt;
  if (!fits) {
    size_t fr = 0, tot = 0;
    GPF_HIP(c, hipMemGetInfo(&fr, &tot));
    const int64_t per_col = (Np + 2 * c->nt) * 8;
    const int64_t maxcols = std::max<int64_t>(T, (int64_t)((double)fr * 0.5 / (double)per_col));
    chunk = std::min<int64_t>(chunk, maxcols);
    Cp = ((chunk + T - 1) / T) * T;
  }
  // buffers kept from the previous call when they are large enough (a hipMalloc/hipFree of the
  // Np x Cp cross-covariance per call cost ~1 ms of the call's wall time); pinned host staging
  // for the query coordinates and the outputs (pageable copies stage through a bounce buffer)
  if (c->p_cols < Cp || c->p_np != Np || c->p_d != c->d || c->p_nt != c->nt) {
    GPF_HIP(c, hipStreamSynchronize(c->stream));
    free_pred(c);
    GPF_HIP(c, hipMalloc(&c->p_xf, (size_t)c->d * Cp * 8));
    GPF_HIP(c, hipMalloc(&c->p_ks, (size_t)Np * Cp * 8));
    GPF_HIP(c, hipMalloc(&c->p_vsq, (size_t)c->nt * Cp * 8));
    GPF_HIP(c, hipMalloc(&c->p_vz, (size_t)c->nt * Cp * 8));
    GPF_HIP(c, hipMalloc(&c->p_mu, (size_t)Cp * 8));
    GPF_HIP(c, hipMalloc(&c->p_sd, (size_t)Cp * 8));
    GPF_HIP(c, hipHostMalloc((void**)&c->p_hx, (size_t)c->d * Cp * 8, hipHostMallocDefault));
    GPF_HIP(c, hipHostMalloc((void**)&c->p_hout, (size_t)2 * Cp * 8, hipHostMallocDefault));
    c->p_cols = Cp;
    c->p_np = Np;
    c->p_d = c->d;
    c->p_nt = c->nt;
  }
  // (Two overlaps of V = U K_s with the single-particle factorisation were built and measured in
  // round 4 — V's row tiles on a low-priority side stream behind each factor launch, and the same
  // with the CUs partitioned by stream CU masks — and removed: the factorisation's latency-bound
  // chain needs the whole chip, profiles/r4/ab_r4g_summary.txt, ab_pred_cumask.txt.)
  double *d_xf = c->p_xf, *d_ks = c->p_ks, *d_vsq = c->p_vsq, *d_vz = c->p_vz, *d_mu = c->p_mu, *d_sd = c->p_sd;
  double* hx = c->p_hx;
  const double* d_z = c->d_yb;  // z = U y of particle slot 0
  auto stage_chunk = [&](int64_t s0, int64_t m) -> int {
    for (int k = 0; k < c->d; ++k) std::memcpy(hx + (size_t)k * Cp, xfit + (size_t)k * M + s0, (size_t)m * 8);
    GPF_HIP(c, hipMemcpyAsync(d_xf, hx, (size_t)c->d * Cp * 8, hipMemcpyHostToDevice, c->stream));
    return GPF_OK;
  };
  // the length scales and chunk 0's coordinates first, then the factorisation
  std::memcpy(c->h_ls, ls, (size_t)c->d * 8);
  GPF_HIP(c, hipMemcpyAsync(c->d_ls, c->h_ls, (size_t)c->d * 8, hipMemcpyHostToDevice, c->stream));
  int rc = stage_chunk(0, std::min<int64_t>(chunk, M));
  if (rc) return rc;
  rc = factor_single_async(c, nullptr, nullptr);
  if (rc) return rc;
  for (int64_t s = 0; s < M && rc == GPF_OK; s += chunk) {
    const int64_t m = std::min<int64_t>(chunk, M - s);
    const int nqt = (int)((m + T - 1) / T);
    const int Cm = nqt * T;
    if (s > 0) {
      if (hipStreamSynchronize(c->stream) != hipSuccess) {  // the staging buffer is reused
        rc = GPF_HIP_ERROR;
        break;
      }
      if ((rc = stage_chunk(s, m))) break;
    }
    rc = launch(c, PC_PREDK, 8.0 * Np * Cm, [&] {
      gpf::launch_cross_cov(c->stream, (int)c->N, (int)m, (int)Np, Cm, c->d, c->d_x, (int)c->N, d_xf, (int)Cp, c->d_ls,
                            d_ks, (int64_t)Cp);
    });
    if (rc) break;
    // V = U K_s over every row tile of U (row tile t has t+1 column tiles, the last triangular)
    const double vflops = 2.0 * T * T * (double)Cm * ((double)c->nt * (c->nt + 1) / 2) - (double)T * T * Cm * c->nt;
    rc = launch(c, PC_PRED, vflops, [&] {
      hipLaunchKernelGGL(gpf::k_predict_vsq, dim3(nqt, c->nt), dim3(gpf::Geo<T>::NTH), 0, c->stream, (int)Np, c->d_U,
                         d_ks, (int)Cp, d_vsq, d_z, d_vz, 0);
    });
    if (rc) break;
    rc = launch(c, PC_LOSS, 0.0, [&] {
      hipLaunchKernelGGL(gpf::k_predict_out, dim3((unsigned)((m + NTHR - 1) / NTHR)), dim3(NTHR), 0, c->stream, c->nt,
                         (int)m, d_vz, (int)Cp, d_vsq, d_mu, d_sd);
    });
    if (rc) break;
    if (hipMemcpyAsync(c->p_hout, d_mu, (size_t)m * 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipMemcpyAsync(c->p_hout + Cp, d_sd, (size_t)m * 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
      rc = GPF_HIP_ERROR;
      c->err = "gpf_predict: copy back failed";
      break;
    }
    if (s == 0) {  // the factorisation's status (its copy preceded this synchronisation)
      rc = factor_status(c);
      if (rc) break;
    }
    std::memcpy(mu + s, c->p_hout, (size_t)m * 8);
    std::memcpy(sd + s, c->p_hout + Cp, (size_t)m * 8);
  }
  hipStreamSynchronize(c->stream);
  if (c->prof) harvest(c);
  // keep the query-chunk buffers for the next call only while they are modest (a huge batch_size
  // can size them up to half of free HBM; see keep_bytes)
  if ((double)c->p_np * (double)c->p_cols * 8.0 > keep_bytes()) free_pred(c);
  return rc;
}

// ---- KMeans subsample (find_len_scales.py:25-47; gpf_kmeans.hip) ----
int gpf_kmeans_set(gpf_ctx* c, const double* X, int64_t n, int d) {
  if (!c) return GPF_BAD_ARG;
  if (n <= 0 || d <= 0 || d > gpf::DMAX || !X) return bad_arg(c, "gpf_kmeans_set: bad arguments");
  hipSetDevice(c->device);
  GPF_HIP(c, hipStreamSynchronize(c->stream));
  if (n != c->km_n || d != c->km_d) {
    hipFree(c->km_x); hipFree(c->km_dist); hipFree(c->km_lab);
    c->km_x = c->km_dist = nullptr;
    c->km_lab = nullptr;
    c->km_n = 0;
    GPF_HIP(c, hipMalloc(&c->km_x, (size_t)n * d * 8));
    GPF_HIP(c, hipMalloc(&c->km_dist, (size_t)n * 8));
    GPF_HIP(c, hipMalloc(&c->km_lab, (size_t)n * 4));
    c->km_n = n;
    c->km_d = d;
  }
  GPF_HIP(c, hipMemcpyAsync(c->km_x, X, (size_t)n * d * 8, hipMemcpyHostToDevice, c->stream));
  GPF_HIP(c, hipStreamSynchronize(c->stream));
  return GPF_OK;
}

int gpf_kmeans_step(gpf_ctx* c, const double* centers, int k, int update, int* labels, double* sums,
                    double* counts, double* dist) {
  if (!c) return GPF_BAD_ARG;
  if (c->km_n <= 0) return bad_arg(c, "gpf_kmeans_step: call gpf_kmeans_set first");
  const int d = c->km_d;
  if (k <= 0 || !centers || !labels || (update && (!sums || !counts))) return bad_arg(c, "gpf_kmeans_step: bad arguments");
  if ((int64_t)k * (d + 1) > gpf::KM_MAXKD)  // centres + norms in LDS (gpfit.kmeans falls back to the host fit)
    return bad_arg(c, "gpf_kmeans_step: k x (d + 1) exceeds KM_MAXKD (8192)");
  hipSetDevice(c->device);
  if (k > c->km_kcap || d != c->km_cd) {  // the centre buffers are k x d: both sizes matter
    GPF_HIP(c, hipStreamSynchronize(c->stream));
    hipFree(c->km_c); hipFree(c->km_sums); hipFree(c->km_cnt);
    c->km_c = c->km_sums = c->km_cnt = nullptr;
    c->km_kcap = 0;
    GPF_HIP(c, hipMalloc(&c->km_c, (size_t)k * d * 8));
    GPF_HIP(c, hipMalloc(&c->km_sums, (size_t)k * d * 8));
    GPF_HIP(c, hipMalloc(&c->km_cnt, (size_t)k * 8));
    c->km_kcap = k;
    c->km_cd = d;
  }
  const int64_t n = c->km_n;
  GPF_HIP(c, hipMemcpyAsync(c->km_c, centers, (size_t)k * d * 8, hipMemcpyHostToDevice, c->stream));
  gpf::launch_km_assign(c->stream, n, d, k, c->km_x, c->km_c, c->km_lab, c->km_dist);
  GPF_HIP(c, hipGetLastError());
  if (update) {
    hipLaunchKernelGGL(gpf::k_km_sums, dim3((unsigned)k), dim3(NTHR), 0, c->stream, n, d, c->km_x, c->km_lab, c->km_sums,
                       c->km_cnt);
    GPF_HIP(c, hipGetLastError());
    GPF_HIP(c, hipMemcpyAsync(sums, c->km_sums, (size_t)k * d * 8, hipMemcpyDeviceToHost, c->stream));
    GPF_HIP(c, hipMemcpyAsync(counts, c->km_cnt, (size_t)k * 8, hipMemcpyDeviceToHost, c->stream));
  }
  GPF_HIP(c, hipMemcpyAsync(labels, c->km_lab, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
  if (dist) GPF_HIP(c, hipMemcpyAsync(dist, c->km_dist, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
  GPF_HIP(c, hipStreamSynchronize(c->stream));
  return GPF_OK;
}

int gpf_kernel(gpf_ctx* c, const double* x1, int64_t N1, const double* x2, int64_t N2, int d, const double* l,
               double* out) {
  if (!c) return GPF_BAD_ARG;
  if (N1 < 0 || N2 < 0 || d <= 0 || d > gpf::DMAX || !l) return bad_arg(c, "gpf_kernel: bad arguments");
  if (N1 == 0 || N2 == 0) return GPF_OK;
  if (!x1 || !x2 || !out) return bad_arg(c, "gpf_kernel: null buffer");
  hipSetDevice(c->device);
  double *dx1 = nullptr, *dx2 = nullptr, *dl = nullptr, *dout = nullptr;
  GPF_HIP(c, hipMalloc(&dx1, (size_t)N1 * d * 8));
  GPF_HIP(c, hipMalloc(&dx2, (size_t)N2 * d * 8));
  GPF_HIP(c, hipMalloc(&dl, (size_t)d * 8));
  GPF_HIP(c, hipMalloc(&dout, (size_t)N1 * N2 * 8));
  GPF_HIP(c, hipMemcpyAsync(dx1, x1, (size_t)N1 * d * 8, hipMemcpyHostToDevice, c->stream));
  GPF_HIP(c, hipMemcpyAsync(dx2, x2, (size_t)N2 * d * 8, hipMemcpyHostToDevice, c->stream));
  GPF_HIP(c, hipMemcpyAsync(dl, l, (size_t)d * 8, hipMemcpyHostToDevice, c->stream));
  int rc = launch(c, PC_BUILD, 8.0 * N1 * N2, [&] {
    gpf::launch_cross_cov(c->stream, (int)N1, (int)N2, (int)N1, (int)N2, d, dx1, (int)N1, dx2, (int)N2, dl, dout, (int64_t)N2);
  });
  if (rc == GPF_OK) {
    if (hipMemcpyAsync(out, dout, (size_t)N1 * N2 * 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
      rc = GPF_HIP_ERROR;
      c->err = "gpf_kernel: copy back failed";
    }
  }
  if (c->prof) harvest(c);
  hipFree(dx1); hipFree(dx2); hipFree(dl); hipFree(dout);
  return rc;
}

int gpf_log_marginal_likelihood(gpf_ctx* c, const double* ls, double* out) {
  if (!c || !ls || !out) return GPF_BAD_ARG;
  if (c->N <= 0) return bad_arg(c, "gpf_log_marginal_likelihood: call gpf_set_data first");
  hipSetDevice(c->device);
  if (c->K <= 0) c->K = 2;
  double* alpha = nullptr;
  int rc = factor_single(c, ls, &alpha);
  if (rc) return rc;
  const int64_t N = c->N, Np = c->Npad;
  std::vector<double> a(N), dg(N);
  GPF_HIP(c, hipMemcpy(a.data(), alpha, (size_t)N * 8, hipMemcpyDeviceToHost));
  GPF_HIP(c, hipMemcpy2D(dg.data(), 8, c->d_L, (size_t)(Np + 1) * 8, 8, (size_t)N, hipMemcpyDeviceToHost));
  double ya = 0.0, ld = 0.0;
  for (int64_t i = 0; i < N; ++i) ya += c->h_y[i] * a[i];
  for (int64_t i = 0; i < N; ++i) ld += std::log(dg[i]);
  *out = -0.5 * ya - ld - 0.5 * (double)N * std::log(2.0 * M_PI);
  return GPF_OK;
}

static int plan_fail(char* msg, int len, const char* fmt, ...) {
  if (msg && len > 0) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(msg, (size_t)len, fmt, ap);
    va_end(ap);
  }
  return GPF_BAD_ARG;
}

// Host-only structural check of the k_step dispatch plan (no device, no context): see gpfit.h.
// The persistent factorisation's queues (gpf::p_decode, as k_factor decodes its tickets): every
// (block column, particle, tile) exactly once, one SYRK item per particle for 1 <= J <= nt-2, every
// particle in one queue, and each item's inputs (the counters it waits for) produced by items
// earlier in that queue — the deadlock-freedom argument of gpf_persist.hip.
static int persist_check(int pc, int nt, long long* stats, char* msg, int msg_len) {
  const int nq = gpf::p_nq(pc);
  // done[p][...]: the ticket position at which each counter value first becomes available
  std::vector<long long> seen((size_t)pc * nt * nt, 0), syrk((size_t)pc * nt, 0);
  std::vector<int> lcol((size_t)pc * nt, 0), ucol((size_t)pc * nt, 0), sdone((size_t)pc * nt, 0);
  for (int p = 0; p < pc; ++p) ucol[(size_t)p * nt] = 1;  // k_diag before the launch
  long long items = 0, tiles = 0, syrks = 0;
  for (int q = 0; q < nq; ++q) {
    const long long n = gpf::p_queue_items(pc, nt, q);
    int Jc = 0;
    long long bc = 0;
    for (long long t = 0; t < n; ++t) {
      int p = -1, w = -2;
      const int kind = gpf::p_decode(t, pc, nt, q, Jc, bc, p, w);
      const int J = Jc;
      if (p < 0 || p >= pc || p % nq != q || J < 0 || J >= nt)
        return plan_fail(msg, msg_len, "persistent queue %d ticket %lld decodes out of range (J=%d p=%d)", q, t, J, p);
      int* lc = &lcol[(size_t)p * nt];
      int* uc = &ucol[(size_t)p * nt];
      int* sd = &sdone[(size_t)p * nt];
      // items run in ticket order here: a wait that is not yet satisfied would wait for a later item
      if (kind == gpf::PK_SYRK) {
        if (!gpf::p_sy(J, nt) || syrk[(size_t)p * nt + J]++)
          return plan_fail(msg, msg_len, "persistent: misplaced or duplicate SYRK item J=%d p=%d", J, p);
        if (lc[J + 1] < J) return plan_fail(msg, msg_len, "persistent: SYRK J=%d p=%d before its row", J, p);
        sd[J + 1] = 1;
        ++syrks;
      } else {
        if (w < 0 || w >= nt - 1) return plan_fail(msg, msg_len, "persistent: tile %d out of range (J=%d)", w, J);
        long long& cnt = seen[((size_t)p * nt + J) * nt + w];
        if (cnt++) return plan_fail(msg, msg_len, "persistent: tile J=%d p=%d w=%d twice", J, p, w);
        if (kind == gpf::PK_LTILE) {
          const int I = J + 1 + w;
          if ((J > 0 && (lc[I] < J || lc[J] < J)) || uc[J] < J + 1 || (I == J + 1 && J > 0 && !sd[I]))
            return plan_fail(msg, msg_len, "persistent: L tile (%d, %d) of p=%d ahead of its inputs", J, I, p);
          if (lc[I] != J) return plan_fail(msg, msg_len, "persistent: row %d of p=%d out of order", I, p);
          lc[I] = J + 1;
          if (I == J + 1) uc[I] = I + 1;  // the critical tile factors block I
        } else {
          const int K = w - (nt - 1 - J);
          if (K < 0 || K >= J || lc[J] < J || uc[K] < J || uc[J] < J + 1)
            return plan_fail(msg, msg_len, "persistent: U tile (%d, %d) of p=%d ahead of its inputs", J, K, p);
          if (uc[K] != J) return plan_fail(msg, msg_len, "persistent: U column %d of p=%d out of order", K, p);
          uc[K] = J + 1;
        }
        ++tiles;
      }
      ++items;
    }
  }
  for (int p = 0; p < pc; ++p)
    for (int J = 0; J < nt; ++J) {
      if (syrk[(size_t)p * nt + J] != gpf::p_sy(J, nt))
        return plan_fail(msg, msg_len, "persistent: particle %d column %d has %lld SYRK items", p, J, syrk[(size_t)p * nt + J]);
      for (int w = 0; w < nt - 1; ++w)
        if (seen[((size_t)p * nt + J) * nt + w] != 1)
          return plan_fail(msg, msg_len, "persistent: tile J=%d p=%d w=%d run %lld times", J, p, w,
                           seen[((size_t)p * nt + J) * nt + w]);
    }
  if (stats) {
    stats[0] = 1;
    stats[1] = items;
    stats[2] = tiles;
    stats[3] = 0;
    stats[4] = 1;
    stats[5] = 1;
    stats[6] = 1;
    stats[7] = 0;
    stats[8] = syrks;
    stats[9] = 1;
    stats[10] = 0;
  }
  return GPF_OK;
}

int gpf_plan_check(int pc, int nt, long long* stats, char* msg, int msg_len) {
  if (msg && msg_len > 0) msg[0] = 0;
  if (pc <= 0 || nt <= 0) return plan_fail(msg, msg_len, "bad arguments pc=%d nt=%d", pc, nt);
  if (persist_on(pc, nt)) return persist_check(pc, nt, stats, msg, msg_len);
  int S = 1, Smax = 1;
  split_sizes(pc, nt, S, Smax);
  std::vector<StepLaunch> plan;
  step_plan(pc, nt, S, Smax, plan);
  const int ntl = nt - 1, ng = num_groups(pc, nt);
  const size_t part_cap = Smax > 1 ? (size_t)pc * ntl * Smax * T * T : 0;
  const size_t cstride = (size_t)gpf::split_cnt_stride(nt), cnt_cap = Smax > 1 ? (size_t)pc * ntl * cstride : 0;
  // partial-slot and counter ranges each group touches: groups run concurrently, so they must
  // be disjoint (within a group the launches are ordered on its stream)
  std::vector<size_t> plo(MAX_GROUPS, SIZE_MAX), phi(MAX_GROUPS, 0), clo(MAX_GROUPS, SIZE_MAX), chi(MAX_GROUPS, 0);
  long long wgs = 0, whole_tiles = 0, split_tiles = 0;
  std::vector<int> whole, piece, diag, syrk;
  long long diag_wgs = 0, syrk_wgs = 0;
  std::vector<int> la_prev(MAX_GROUPS, 0), pair_prev(MAX_GROUPS, 0), pairJ(MAX_GROUPS, -1), lall_prev(MAX_GROUPS, 0);
  const int lsmax = lall_smax(nt);
  if ((int)plan.size() != (nt > 1 ? nt * ng : 0)) return plan_fail(msg, msg_len, "plan has %d launches, want %d",
                                                              (int)plan.size(), nt * ng);
  for (const StepLaunch& l : plan) {
    if (l.gc <= 0 || l.p0 < 0 || l.p0 + l.gc > pc || l.g < 0 || l.g >= ng)
      return plan_fail(msg, msg_len, "J=%d: bad group range p0=%d gc=%d g=%d", l.J, l.p0, l.gc, l.g);
    if (l.S < 1 || (l.split == gpf::SPLIT_NONE && (l.S != 1 || l.S2 != 1)) || (l.split == gpf::SPLIT_ALL && l.S2 != Smax))
      return plan_fail(msg, msg_len, "J=%d g=%d: split kind %d with S=%d S2=%d", l.J, l.g, l.split, l.S, l.S2);
    if (l.split != gpf::SPLIT_NONE && Smax < 2)
      return plan_fail(msg, msg_len, "J=%d g=%d: split launch without split-K buffers (Smax=%d)", l.J, l.g, Smax);
    // the look-ahead partial a seeded launch reads (slot of J-1) is never the one it writes (slot of J)
    if ((l.la & 2) && (l.la & 1) && gpf::la_slot(0, l.J - 1) == gpf::la_slot(0, l.J))
      return plan_fail(msg, msg_len, "J=%d g=%d: look-ahead reads and writes the same slot", l.J, l.g);
    const int tiles = l.gc * ntl;
    auto pieces_of = [&](int w) { return l.split == gpf::SPLIT_ALL ? gpf::split_all_pieces(l.J, w, nt, l.S) : l.S; };
    for (int w = 0; w < ntl; ++w)
      if (pieces_of(w) > l.S2) return plan_fail(msg, msg_len, "J=%d tile %d: %d pieces but %d slots", l.J, w, pieces_of(w), l.S2);
    whole.assign((size_t)tiles, 0);
    piece.assign((size_t)tiles * l.S2, 0);
    diag.assign((size_t)l.gc, 0);
    syrk.assign((size_t)l.gc, 0);
    if (l.sy && (!l.defer || l.J < 1 || l.J > nt - 2 || l.split == gpf::SPLIT_ALL))
      return plan_fail(msg, msg_len, "J=%d: SYRK workgroups without a diagonal block to reduce", l.J);
    if (l.defer && l.split == gpf::SPLIT_ALL)
      return plan_fail(msg, msg_len, "J=%d: deferred diagonal update under the all-tile split", l.J);
    // the flat finish waits for the diagonal block inside the launch (gpf::flat_piece)
    if (l.split == gpf::SPLIT_ALL && !l.ed)
      return plan_fail(msg, msg_len, "J=%d: all-tile split launch without the early diagonal factor", l.J);
    // look-ahead: LA workgroups only where a next critical tile exists, no split, early diagonal
    // factor; a seeded launch follows a launch of the same group that ran them
    if (l.la && (l.split != gpf::SPLIT_NONE || !l.ed || ((l.la & 1) && (l.J < 1 || l.J > nt - 3)) ||
                 ((l.la & 2) && (l.J < 2 || l.J > nt - 2 || !(la_prev[l.g] & 1)))))
      return plan_fail(msg, msg_len, "J=%d g=%d: look-ahead bits %d out of place", l.J, l.g, l.la);
    if ((la_prev[l.g] & 1) && !(l.la & 2))
      return plan_fail(msg, msg_len, "J=%d g=%d: look-ahead partials of launch J-1 left unused", l.J, l.g);
    la_prev[l.g] = l.la;
    if (l.ro && (ng != 1 || !l.ed || !l.sy || l.split != gpf::SPLIT_NONE || l.grp != 0 || l.J < 1 || 3 * l.gc > 256 ||
                 l.grid != (unsigned)(l.gc * (nt - 1) + 2 * l.gc)))
      return plan_fail(msg, msg_len, "J=%d g=%d: reordered dispatch out of place", l.J, l.g);
    // paired block columns: a lead launch (J odd, with a block column behind it, fused diagonal factor,
    // deferred update, no split, groups of 8 particles) is followed on its stream by the follow
    // launch J+1, and only there
    // all-tile look-ahead (early-diagonal launches, l.pair bits): pieces only from J >= 1 with a block
    // column behind, consumed by the next launch of the same group (which reads the other parity)
    if (l.ed && l.pair) {
      if (l.split != gpf::SPLIT_NONE || !l.defer || (l.la & 1) || ((l.la & 2) && (l.pair & 2)) || l.ro || nt < 4 ||
          ((l.pair & 1) && gpf::lall_items(l.J, nt) == 0) ||
          ((l.pair & 2) && (l.J < 2 || !(lall_prev[l.g] & 1) || pairJ[l.g] != l.J - 1)))
        return plan_fail(msg, msg_len, "J=%d g=%d: look-ahead pieces %d out of place", l.J, l.g, l.pair);
    }
    if ((lall_prev[l.g] & 1) && !(l.ed && (l.pair & 2)))
      return plan_fail(msg, msg_len, "J=%d g=%d: launch J-1's look-ahead pieces left unused", l.J, l.g);
    lall_prev[l.g] = l.ed ? l.pair : 0;
    if (!l.ed && l.pair && (l.split != gpf::SPLIT_NONE || !l.defer || l.grp != 0 || l.gc % 8 != 0 || nt < 4 ||
                   (l.pair == 1 && (!(l.J & 1) || l.J + 1 > nt - 1 || !l.sy)) ||
                   (l.pair == 2 && (l.sy || pair_prev[l.g] != 1 || pairJ[l.g] != l.J - 1))))
      return plan_fail(msg, msg_len, "J=%d g=%d: paired block column %d out of place", l.J, l.g, l.pair);
    if (pair_prev[l.g] == 1 && l.pair != 2)
      return plan_fail(msg, msg_len, "J=%d g=%d: the lead launch's partials left unused", l.J, l.g);
    pair_prev[l.g] = l.ed ? 0 : l.pair;
    pairJ[l.g] = l.J;
    if (!l.ed && l.pair == 1) {
      if (l.grid != (unsigned)(l.gc * gpf::pair_grid_per_particle(l.J, nt)))
        return plan_fail(msg, msg_len, "J=%d g=%d: lead launch grid %u", l.J, l.g, l.grid);
      std::vector<int> pla((size_t)tiles, 0), syp((size_t)l.gc, 0);
      for (unsigned b = 0; b < l.grid; ++b) {
        int p = -1, w = -1;
        const int role = gpf::pair_decode((int)b, l.J, l.gc, nt, p, w);
        if (p < 0 || p >= l.gc || (int)(b & 7) != (p & 7))
          return plan_fail(msg, msg_len, "J=%d block %u: pair decode p=%d (its XCD is not the particle's)", l.J, b, p);
        if (role != gpf::ROLE_WHOLE) {  // a partner: its tile's workgroup of the same particle 8 or 16 ids
          // earlier (a SYRK workgroup: its critical tile, which waits for it, 8 ids later)
          int p2 = -1, w2 = -1, ok = 0;
          for (int k = 1; k <= 2 && !ok; ++k) {
            const int b2 = role == gpf::ROLE_SYRK ? (int)b + 8 * k : (int)b - 8 * k;
            ok = b2 >= 0 && b2 < (int)l.grid && gpf::pair_decode(b2, l.J, l.gc, nt, p2, w2) == gpf::ROLE_WHOLE &&
                 p2 == p && w2 == (role == gpf::ROLE_SYRK ? 0 : w) && (role != gpf::ROLE_SYRK || k == 1);
          }
          if (!ok) return plan_fail(msg, msg_len, "J=%d block %u: partner (role %d) not beside its tile", l.J, b, role);
        }
        if (role == gpf::ROLE_SYRK) {
          if (syrk[p]++) return plan_fail(msg, msg_len, "J=%d: duplicate SYRK workgroup p=%d", l.J, p);
        } else if (role == gpf::ROLE_SYRKP) {
          if (w != 1 || l.J + 2 > nt - 1 || syp[p]++)
            return plan_fail(msg, msg_len, "J=%d: misplaced or duplicate partial SYRK p=%d", l.J, p);
        } else if (role == gpf::ROLE_PLA) {
          if (w < 1 || w >= ntl || pla[(size_t)p * ntl + w]++)
            return plan_fail(msg, msg_len, "J=%d: misplaced or duplicate look-ahead partial p=%d w=%d", l.J, p, w);
          if (gpf::pair_slot(p, w - 1, nt) + (size_t)T * T > (size_t)l.gc * ntl * T * T)
            return plan_fail(msg, msg_len, "J=%d: partial slot outside the group's buffer", l.J);
        } else if (role == gpf::ROLE_WHOLE) {
          if (w < 0 || w >= ntl) return plan_fail(msg, msg_len, "J=%d block %u decodes out of range", l.J, b);
          ++whole[(size_t)p * ntl + w];
        } else {
          return plan_fail(msg, msg_len, "J=%d block %u: role %d in a lead launch", l.J, b, role);
        }
        ++wgs;
      }
      for (int q = 0; q < l.gc; ++q) {
        if (syrk[q] != 1 || syp[q] != (l.J + 2 <= nt - 1 ? 1 : 0))
          return plan_fail(msg, msg_len, "J=%d particle %d: %d SYRK, %d partial SYRK workgroups", l.J, q, syrk[q], syp[q]);
        syrk_wgs += 1;
        for (int w = 0; w < ntl; ++w) {
          if (whole[(size_t)q * ntl + w] != 1 || pla[(size_t)q * ntl + w] != (w >= 1 ? 1 : 0))
            return plan_fail(msg, msg_len, "J=%d particle %d tile %d: %d runs, %d partials", l.J, q, w,
                             whole[(size_t)q * ntl + w], pla[(size_t)q * ntl + w]);
          ++whole_tiles;
        }
      }
      continue;
    }
    std::vector<int> lawg((size_t)l.gc, 0);
    const int nstd = (l.ed ? l.gc : 0) + (l.sy ? l.gc : 0) + l.gc * ntl;
    const int lpb = lall_pb(), ltag = gpf::lall_tag(l.gc, lpb, lsmax);
    std::vector<int> lpc;
    if (l.ed && (l.pair & 1)) {
      if (l.grid != (unsigned)(nstd + l.gc * gpf::lall_total(l.J, nt, lpb)))
        return plan_fail(msg, msg_len, "J=%d g=%d: look-ahead launch grid %u", l.J, l.g, l.grid);
      lpc.assign((size_t)l.gc * lsmax, 0);
    }
    for (unsigned b = 0; b < l.grid; ++b) {
      int p = -1, w = -1, sidx = -1;
      if (l.ed && (l.pair & 1) && gpf::lall_is_piece((int)b, l.J, l.gc, nt, nstd, l.pair, ltag)) {
        // a look-ahead piece: every (particle, item, piece) once
        int it = -1;
        gpf::lall_decode(gpf::lall_piece_index((int)b, l.gc, nt, nstd, l.pair), l.J, l.gc, nt, lpb, p, it, sidx);
        if (p < 0 || p >= l.gc || it < 0 || it >= gpf::lall_items(l.J, nt) || sidx < 0 || sidx >= gpf::lall_np(l.J, it, nt, lpb))
          return plan_fail(msg, msg_len, "J=%d block %u: look-ahead piece decodes out of range", l.J, b);
        const int o = gpf::lall_off(l.J, it, nt, lpb) + sidx;
        if (o >= lsmax || gpf::lall_slot(l.J, it, sidx, p, l.gc, nt, lsmax, lpb) + (size_t)T * T > (size_t)2 * l.gc * lsmax * T * T ||
            lpc[(size_t)p * lsmax + o]++)
          return plan_fail(msg, msg_len, "J=%d block %u: look-ahead piece slot %d duplicate or outside", l.J, b, o);
        ++wgs;
        continue;
      }
      // (pieces ahead of the tiles: the block index the kernel hands step_decode)
      const unsigned bt = (l.ed && (l.pair & 5) == 5) ? (unsigned)gpf::lall_tile_block((int)b, l.J, l.gc, nt, nstd, ltag) : b;
      const int role =
          l.split == gpf::SPLIT_ALL ? gpf::step_decode<gpf::SPLIT_ALL>(bt, l.J, l.gc, nt, l.grp, l.S, l.ed, 0, 0, p, w, sidx)
                                    : gpf::step_decode<gpf::SPLIT_NONE>(bt, l.J, l.gc, nt, l.grp, l.S, l.ed, l.sy,
                                                                        (l.la & 1) && !l.sy, p, w, sidx, l.ro);
      if (role == gpf::ROLE_DIAG) {  // one diagonal workgroup per particle, ahead of every tile of the launch
        // (reordered: right behind the particles' light U tiles, which wait for it, and the SYRK workgroups)
        if (!l.ed || p < 0 || p >= l.gc || (unsigned)p + (l.ro ? 2 * l.gc : 0) != bt || diag[p]++)
          return plan_fail(msg, msg_len, "J=%d block %u: misplaced or duplicate diagonal workgroup (p=%d)", l.J, b, p);
        ++wgs;
        continue;
      }
      if (role == gpf::ROLE_LA) {  // one per particle, right behind the diagonal and SYRK workgroups
        if (!(l.la & 1) || l.sy || p < 0 || p >= l.gc || (unsigned)p + (l.ed ? l.gc : 0) != bt || lawg[p]++)
          return plan_fail(msg, msg_len, "J=%d block %u: misplaced or duplicate look-ahead workgroup (p=%d)", l.J, b, p);
        ++wgs;
        continue;
      }
      if (role == gpf::ROLE_SYRK) {  // one per particle, right behind the diagonal workgroups (reordered: the light U tiles)
        if (!l.sy || p < 0 || p >= l.gc || (unsigned)p + (l.ro || l.ed ? l.gc : 0) != bt || syrk[p]++)
          return plan_fail(msg, msg_len, "J=%d block %u: misplaced or duplicate SYRK workgroup (p=%d)", l.J, b, p);
        ++wgs;
        continue;
      }
      if (p < 0 || p >= l.gc || w < 0 || w >= ntl || sidx < 0 || sidx >= pieces_of(w))
        return plan_fail(msg, msg_len, "J=%d block %u decodes out of range (p=%d w=%d)", l.J, b, p, w);
      const int t = p * ntl + w;
      if (role == gpf::ROLE_WHOLE) {
        ++whole[t];
      } else if (role == gpf::ROLE_PIECE) {
        if (pieces_of(w) < 2) return plan_fail(msg, msg_len, "J=%d block %u is a piece of an unsplit tile", l.J, b);
        ++piece[(size_t)t * l.S2 + sidx];
        // slots as k_step addresses them: S2 per tile
        // counters: the flat finish's FLAT_CNT words of (particle, launch, tile) inside the
        // particle's ntl * cstride (gpf::flat_piece)
        const size_t off = l.part_off + ((size_t)t * l.S2 + sidx) * T * T;
        const size_t ci = l.cnt_off + (size_t)p * ntl * cstride + ((size_t)l.J * ntl + w) * gpf::FLAT_CNT;
        const size_t cn = gpf::FLAT_CNT;
        if (off + (size_t)T * T > part_cap || ci + cn > cnt_cap || l.S2 > gpf::SPLIT_MAXS ||
            ci + cn > l.cnt_off + (size_t)(p + 1) * ntl * cstride)
          return plan_fail(msg, msg_len, "J=%d tile %d piece %d outside the split buffers (S=%d S2=%d)", l.J, t, sidx, l.S,
                           l.S2);
        plo[l.g] = std::min(plo[l.g], off);
        phi[l.g] = std::max(phi[l.g], off + (size_t)T * T);
        clo[l.g] = std::min(clo[l.g], ci);
        chi[l.g] = std::max(chi[l.g], ci + cn);
      }
      ++wgs;
    }
    for (size_t i = 0; i < lpc.size(); ++i)
      if ((int)(i % lsmax) < gpf::lall_total(l.J, nt, lpb) && lpc[i] != 1)
        return plan_fail(msg, msg_len, "J=%d particle %d: look-ahead piece %d run %d times", l.J, (int)(i / lsmax),
                         (int)(i % lsmax), lpc[i]);
    for (int q = 0; q < l.gc; ++q) {
      if (diag[q] != l.ed) return plan_fail(msg, msg_len, "J=%d particle %d: %d diagonal workgroups", l.J, q, diag[q]);
      diag_wgs += diag[q];
      if (syrk[q] != l.sy) return plan_fail(msg, msg_len, "J=%d particle %d: %d SYRK workgroups", l.J, q, syrk[q]);
      if (lawg[q] != ((l.la & 1) && !l.sy ? 1 : 0))
        return plan_fail(msg, msg_len, "J=%d particle %d: %d look-ahead workgroups", l.J, q, lawg[q]);
      syrk_wgs += syrk[q];
    }
    for (int t = 0; t < tiles; ++t) {
      int np = 0;
      for (int s = 0; s < l.S2; ++s) {
        if (piece[(size_t)t * l.S2 + s] > 1) return plan_fail(msg, msg_len, "J=%d tile %d: piece %d run %d times", l.J, t, s, piece[(size_t)t * l.S2 + s]);
        np += piece[(size_t)t * l.S2 + s];
      }
      if (whole[t] == 1 && np == 0) ++whole_tiles;
      else if (whole[t] == 0 && np == pieces_of(t % ntl)) ++split_tiles;  // S arrivals on a zeroed counter: one finisher
      else return plan_fail(msg, msg_len, "J=%d tile %d: %d whole runs and %d pieces", l.J, t, whole[t], np);
    }
  }
  for (int g = 0; g < ng; ++g)
    if (pair_prev[g] == 1 || (lall_prev[g] & 1)) return plan_fail(msg, msg_len, "group %d ends with unused partials", g);
  for (int a = 0; a < ng; ++a)
    for (int b2 = a + 1; b2 < ng; ++b2) {
      if (plo[a] < phi[a] && plo[b2] < phi[b2] && plo[a] < phi[b2] && plo[b2] < phi[a])
        return plan_fail(msg, msg_len, "groups %d and %d share split-K partial slots", a, b2);
      if (clo[a] < chi[a] && clo[b2] < chi[b2] && clo[a] < chi[b2] && clo[b2] < chi[a])
        return plan_fail(msg, msg_len, "groups %d and %d share split-K counters", a, b2);
    }
  if (stats) {
    stats[0] = (long long)plan.size();
    stats[1] = wgs;
    stats[2] = whole_tiles;
    stats[3] = split_tiles;
    stats[4] = S;
    stats[5] = Smax;
    stats[6] = ng;
    stats[7] = diag_wgs;
    stats[8] = syrk_wgs;
    long long pairs = 0;
    for (const StepLaunch& l : plan) pairs += !l.ed && l.pair == 1;
    stats[9] = 0;      // not persistent
    stats[10] = pairs;  // lead launches (paired block columns)
  }
  return GPF_OK;
}

int gpf_sync(gpf_ctx* c) {
  if (!c) return GPF_BAD_ARG;
  GPF_HIP(c, hipSetDevice(c->device));
  GPF_HIP(c, hipDeviceSynchronize());
  return GPF_OK;
}

int gpf_set_profiling(gpf_ctx* c, int on) {
  if (!c) return GPF_BAD_ARG;
  c->prof = on != 0;  // (profiled batches take the plain launch path, never a graph)
  if (c->prof && !c->d_clk) {
    hipSetDevice(c->device);
    GPF_HIP(c, hipMalloc(&c->d_clk, 2 * sizeof(unsigned long long)));
    GPF_HIP(c, hipMemsetAsync(c->d_clk, 0, 2 * sizeof(unsigned long long), c->stream));
  }
  return GPF_OK;
}

int gpf_reset_profile(gpf_ctx* c) {
  if (!c) return GPF_BAD_ARG;
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  harvest(c);
  std::memset(c->acc, 0, sizeof(c->acc));
  c->evals = 0;
  if (!c->d_clk) GPF_HIP(c, hipMalloc(&c->d_clk, 2 * sizeof(unsigned long long)));
  GPF_HIP(c, hipMemsetAsync(c->d_clk, 0, 2 * sizeof(unsigned long long), c->stream));
  return GPF_OK;
}

int gpf_get_profile(gpf_ctx* c, double* out, int n) {
  if (!c || !out) return 0;
  hipStreamSynchronize(c->stream);
  harvest(c);
  double v[24] = {c->acc[PC_PANEL][0],  c->acc[PC_PANEL][1],  c->acc[PC_PANEL][2], c->acc[PC_DIAG][0],
                  c->acc[PC_DIAG][1],   c->acc[PC_DIAG][2],   c->acc[PC_BUILD][0], c->acc[PC_BUILD][1],
                  c->acc[PC_BUILD][2],  c->acc[PC_LOSS][0],   c->acc[PC_LOSS][1],  c->evals,
                  c->acc[PC_FACTOR][0], c->acc[PC_FACTOR][1], c->acc[PC_FACTOR][2],
                  c->acc[PC_PRED][0],   c->acc[PC_PRED][1],   c->acc[PC_PRED][2],
                  c->acc[PC_PREDK][0],  c->acc[PC_PREDK][1],  c->acc[PC_PREDK][2],
                  c->acc[PC_PSURF][0],  c->acc[PC_PSURF][1],  c->acc[PC_PSURF][2]};
  // [24] shader clock (MHz) the factor kernels held while they ran (gpf::ClockSpan), [25] the
  // device's compute units, [26] the FP64 matrix ceiling at that clock (TFLOP/s, 128 flop per CU
  // per clock)
  unsigned long long clk[2] = {0, 0};
  if (c->d_clk) hipMemcpy(clk, c->d_clk, sizeof(clk), hipMemcpyDeviceToHost);
  const double mhz = clk[1] > 0 ? 100.0 * (double)clk[0] / (double)clk[1] : 0.0;
  const double w[27 - 24] = {mhz, (double)c->ncu, 128.0 * c->ncu * mhz * 1e6 / 1e12};
  const int m = std::min(n, 27);
  for (int i = 0; i < m; ++i) out[i] = i < 24 ? v[i] : w[i - 24];
  return m;
}

int gpf_selftest_mfma(gpf_ctx* c, const double* a, const double* b, double* out) {
  if (!c || !a || !b || !out) return GPF_BAD_ARG;
  hipSetDevice(c->device);
  double *da = nullptr, *db = nullptr, *dc = nullptr;
  GPF_HIP(c, hipMalloc(&da, 64 * 8));
  GPF_HIP(c, hipMalloc(&db, 64 * 8));
  GPF_HIP(c, hipMalloc(&dc, 256 * 8));
  GPF_HIP(c, hipMemcpy(da, a, 64 * 8, hipMemcpyHostToDevice));
  GPF_HIP(c, hipMemcpy(db, b, 64 * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(gpf::k_selftest_mfma, dim3(1), dim3(64), 0, c->stream, da, db, dc);
  GPF_HIP(c, hipGetLastError());
  GPF_HIP(c, hipStreamSynchronize(c->stream));
  GPF_HIP(c, hipMemcpy(out, dc, 256 * 8, hipMemcpyDeviceToHost));
  hipFree(da); hipFree(db); hipFree(dc);
  return GPF_OK;
}

int gpf_debug_factor(gpf_ctx* c, const double* ls, double* L, double* U, double* z, double* alpha) {
  if (!c || !ls || !L || !U || !z || !alpha) return GPF_BAD_ARG;
  if (c->N <= 0) return bad_arg(c, "gpf_debug_factor: call gpf_set_data first");
  hipSetDevice(c->device);
  if (c->K <= 0) c->K = 2;
  double* al = nullptr;
  int rc = factor_single(c, ls, &al);
  if (rc && rc != GPF_NOT_PD) return rc;
  const size_t np = (size_t)c->Npad;
  GPF_HIP(c, hipMemcpy(L, c->d_L, np * np * 8, hipMemcpyDeviceToHost));
  GPF_HIP(c, hipMemcpy(U, c->d_U, np * np * 8, hipMemcpyDeviceToHost));
  GPF_HIP(c, hipMemcpy(z, c->d_yb, np * 8, hipMemcpyDeviceToHost));
  if (al) GPF_HIP(c, hipMemcpy(alpha, al, (size_t)c->N * 8, hipMemcpyDeviceToHost));
  return rc;
}

// Shader clock (MHz) from a ClockSpan buffer: shader clocks over 100 MHz reference clocks.
static double read_clock(const unsigned long long* dclk) {
  unsigned long long h[2] = {0, 0};
  if (hipMemcpy(h, dclk, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess || h[1] == 0) return 0.0;
  return 100.0 * (double)h[0] / (double)h[1];
}

int gpf_bench_clock(gpf_ctx* c, double* mhz) {
  if (!c || !mhz) return GPF_BAD_ARG;
  *mhz = c->bench_sclk;
  return GPF_OK;
}

int gpf_mfma_peak(gpf_ctx* c, int blocks, int iters, double* tflops) {
  if (!c || !tflops || blocks <= 0 || iters <= 0) return GPF_BAD_ARG;
  hipSetDevice(c->device);
  double* out = nullptr;
  GPF_HIP(c, hipMalloc(&out, (size_t)blocks * 8));
  hipEvent_t a, b;
  GPF_HIP(c, hipEventCreate(&a));
  GPF_HIP(c, hipEventCreate(&b));
  unsigned long long* clk = nullptr;
  GPF_HIP(c, hipMalloc(&clk, 2 * sizeof(unsigned long long)));
  GPF_HIP(c, hipMemsetAsync(clk, 0, 2 * sizeof(unsigned long long), c->stream));
  hipLaunchKernelGGL(gpf::k_mfma_rate, dim3(blocks), dim3(NTHR), 0, c->stream, iters, 1.0, out, nullptr);  // warm-up
  GPF_HIP(c, hipEventRecord(a, c->stream));
  hipLaunchKernelGGL(gpf::k_mfma_rate, dim3(blocks), dim3(NTHR), 0, c->stream, iters, 1.0, out, clk);
  GPF_HIP(c, hipEventRecord(b, c->stream));
  GPF_HIP(c, hipEventSynchronize(b));
  c->bench_sclk = read_clock(clk);
  hipFree(clk);
  float ms = 0.f;
  GPF_HIP(c, hipEventElapsedTime(&ms, a, b));
  *tflops = (double)blocks * 4.0 * iters * 8.0 * 2048.0 / (ms * 1e-3) / 1e12;
  hipEventDestroy(a);
  hipEventDestroy(b);
  hipFree(out);
  return GPF_OK;
}

// Probability surface (calc_prob_surf.py:15-30,67-81) of M rows of E tail entries each.
int gpf_prob_surface(gpf_ctx* c, const double* tails, int64_t M, int E, double* y, double* p, int* ok) {
  if (!c) return GPF_BAD_ARG;
  if (M < 0 || E < 0 || E > gpf::PS_EMAX || (M > 0 && (!tails || !y || !p || !ok)))
    return bad_arg(c, "gpf_prob_surface: bad arguments");
  if (M == 0) return GPF_OK;
  hipSetDevice(c->device);
  const int64_t chunk = std::min<int64_t>(M, 1 << 20);
  const int Ea = std::max(E, 1);
  if (c->s_rows < chunk || c->s_e < Ea) {  // grow-only (rows and tail width)
    GPF_HIP(c, hipStreamSynchronize(c->stream));
    free_psurf(c);
    GPF_HIP(c, hipMalloc(&c->s_t, (size_t)chunk * Ea * 8));
    GPF_HIP(c, hipMalloc(&c->s_cmp, (size_t)chunk * Ea * 8));
    GPF_HIP(c, hipMalloc(&c->s_info, (size_t)chunk * sizeof(double4)));
    GPF_HIP(c, hipMalloc(&c->s_y, (size_t)chunk * gpf::PS_POINTS * 8));
    GPF_HIP(c, hipMalloc(&c->s_p, (size_t)chunk * gpf::PS_POINTS * 8));
    GPF_HIP(c, hipMalloc(&c->s_ok, (size_t)chunk * 4));
    c->s_rows = chunk;
    c->s_e = Ea;
  }
  double *dt = c->s_t, *dy = c->s_y, *dp = c->s_p;
  int* dok = c->s_ok;
  int rc = GPF_OK;
  for (int64_t s = 0; s < M && rc == GPF_OK; s += chunk) {
    const int64_t m = std::min<int64_t>(chunk, M - s);
    if (hipMemcpyAsync(dt, tails + s * E, (size_t)m * E * 8, hipMemcpyHostToDevice, c->stream) != hipSuccess) {
      rc = GPF_HIP_ERROR;
      break;
    }
    // algorithmic bytes: the tails read, y and p written, the row flags
    const double bytes = (double)m * (E * 8.0 + 2.0 * gpf::PS_POINTS * 8.0 + 4.0);
    rc = launch(c, PC_PSURF, bytes, [&] {
      hipLaunchKernelGGL(gpf::k_prob_prep, dim3(blocks_for(m)), dim3(NTHR), 0, c->stream, dt, m, E, c->s_cmp, c->s_info);
      hipLaunchKernelGGL(gpf::k_prob_surf, dim3(blocks_for(m * gpf::PS_POINTS)), dim3(NTHR), 0, c->stream, c->s_cmp,
                         c->s_info, m, E, dy, dp, dok);
    });
    if (rc) break;
    if (hipMemcpyAsync(y + s * gpf::PS_POINTS, dy, (size_t)m * gpf::PS_POINTS * 8, hipMemcpyDeviceToHost, c->stream) !=
            hipSuccess ||
        hipMemcpyAsync(p + s * gpf::PS_POINTS, dp, (size_t)m * gpf::PS_POINTS * 8, hipMemcpyDeviceToHost, c->stream) !=
            hipSuccess ||
        hipMemcpyAsync(ok + s, dok, (size_t)m * 4, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
      rc = GPF_HIP_ERROR;
      c->err = "gpf_prob_surface: copy failed";
    }
  }
  if (rc == GPF_HIP_ERROR && c->err.empty()) c->err = "gpf_prob_surface: HIP error";
  hipStreamSynchronize(c->stream);
  if ((double)c->s_rows * (2.0 * c->s_e + 2.0 * gpf::PS_POINTS + 4.5) * 8.0 > keep_bytes()) free_psurf(c);
  return rc;
}

// ---- convex-hull grid fill (convex_hull.py:122-155,203-224; helpers above the C-ABI block) ----
int gpf_hull_fill(gpf_ctx* c, const double* shell, int64_t n, int d, const double* res, const int* decimals,
                  int64_t* m_out) {
  if (!c) return GPF_BAD_ARG;
  if (n <= 0 || d <= 0 || d > gpf::DMAX || !shell || !res || !decimals || !m_out)
    return bad_arg(c, "gpf_hull_fill: bad arguments");
  hipSetDevice(c->device);
  gpf::HullDims hd{};
  hd.d = d;
  for (int j = 0; j < d; ++j) {
    if (!(res[j] > 0.0)) return bad_arg(c, "gpf_hull_fill: resolution must be > 0");
    hd.res[j] = res[j];
    hd.p10[j] = (res[j] < 1.0 && decimals[j] >= 0) ? std::pow(10.0, decimals[j]) : 0.0;
  }
  hipStream_t st = c->stream;
  DevBuf rows;
  GPF_HIP(c, rows.alloc((size_t)n * d * 8, st));
  GPF_HIP(c, hipMemcpyAsync(rows.p, shell, (size_t)n * d * 8, hipMemcpyHostToDevice, st));
  std::vector<int> order(d);
  for (int j = 0; j < d; ++j) order[j] = j;
  int rc = hull_sort_unique(c, rows, n, d, order.data());
  if (rc) return rc;
  for (int i = 0; i < d; ++i) {
    // pass i: the grid is sorted by columns i, i+1, .., i-1 (mod d); fill along the last of them
    hd.axis = (d - 1 + i) % d;
    DevBuf cnt, off, temp, grown;
    GPF_HIP(c, cnt.alloc((size_t)n * 8, st));
    GPF_HIP(c, off.alloc((size_t)n * 8, st));
    hipLaunchKernelGGL(gpf::k_hull_count, dim3(blocks_for(n)), dim3(NTHR), 0, st, rows.as<double>(), n, hd,
                       cnt.as<int64_t>());
    size_t tb = 0;
    GPF_HIP(c, hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt.as<int64_t>(), off.as<int64_t>(), n, st));
    GPF_HIP(c, temp.alloc(std::max<size_t>(tb, 16), st));
    GPF_HIP(c, hipcub::DeviceScan::ExclusiveSum(temp.p, tb, cnt.as<int64_t>(), off.as<int64_t>(), n, st));
    int64_t last[2] = {0, 0};
    GPF_HIP(c, hipMemcpyAsync(&last[0], off.as<int64_t>() + (n - 1), 8, hipMemcpyDeviceToHost, st));
    GPF_HIP(c, hipMemcpyAsync(&last[1], cnt.as<int64_t>() + (n - 1), 8, hipMemcpyDeviceToHost, st));
    GPF_HIP(c, hipStreamSynchronize(st));
    const int64_t add = last[0] + last[1];
    GPF_HIP(c, grown.alloc((size_t)(n + add) * d * 8, st));
    GPF_HIP(c, hipMemcpyAsync(grown.p, rows.p, (size_t)n * d * 8, hipMemcpyDeviceToDevice, st));
    hipLaunchKernelGGL(gpf::k_hull_emit, dim3(blocks_for(n)), dim3(NTHR), 0, st, rows.as<double>(), n, hd,
                       off.as<int64_t>(), grown.as<double>() + (size_t)n * d);
    GPF_HIP(c, hipGetLastError());
    std::swap(rows.p, grown.p);
    n += add;
    for (int j = 0; j < d; ++j) order[j] = (i + 1 + j) % d;
    rc = hull_sort_unique(c, rows, n, d, order.data());
    if (rc) return rc;
  }
  c->hull_rows.resize((size_t)n * d);
  GPF_HIP(c, hipMemcpy(c->hull_rows.data(), rows.p, (size_t)n * d * 8, hipMemcpyDeviceToHost));
  c->hull_d = d;
  *m_out = n;
  return GPF_OK;
}

int gpf_hull_fetch(gpf_ctx* c, double* out) {
  if (!c || !out) return GPF_BAD_ARG;
  if (!c->hull_rows.empty()) std::memcpy(out, c->hull_rows.data(), c->hull_rows.size() * 8);
  return GPF_OK;
}

// Measurement hook: TF/s of the k_step L-tile GEMM core alone (k_gemm_bench) on
// P random Npad x Npad matrices, tiles = workgroups per particle, depth D.
int gpf_gemm_bench(gpf_ctx* c, int mode, int Npad, int P, int tiles, int D, int iters, double* tflops) {
  if (!c || !tflops || Npad % T || D % T || P <= 0 || tiles <= 0 || iters <= 0) return GPF_BAD_ARG;
  if ((D / T + 1 + tiles) * T > Npad) return bad_arg(c, "gpf_gemm_bench: tiles do not fit");
  hipSetDevice(c->device);
  double *L = nullptr, *C = nullptr;
  const size_t n = (size_t)P * Npad * Npad;
  GPF_HIP(c, hipMalloc(&L, n * 8));
  GPF_HIP(c, hipMalloc(&C, (size_t)P * tiles * T * T * 8));
  // mode bit 8: zero operands (rounds 1-3); otherwise hashed values in [-1, 1) (gpf::k_fill_hash);
  // bit 16 / 32: the 3- / 4-stage LDS pipeline (gpf::DenseRun NS) instead of 2
  const auto kb = (mode & 32) ? gpf::k_gemm_bench<4> : (mode & 16) ? gpf::k_gemm_bench<3> : gpf::k_gemm_bench<2>;
  if (mode & 8)
    GPF_HIP(c, hipMemsetAsync(L, 0, n * 8, c->stream));
  else
    hipLaunchKernelGGL(gpf::k_fill_hash, dim3(4096), dim3(NTHR), 0, c->stream, L, (long long)n);
  hipEvent_t a, b;
  GPF_HIP(c, hipEventCreate(&a));
  GPF_HIP(c, hipEventCreate(&b));
  const int W = P * tiles;
  unsigned long long* clk = nullptr;
  GPF_HIP(c, hipMalloc(&clk, 2 * sizeof(unsigned long long)));
  GPF_HIP(c, hipMemsetAsync(clk, 0, 2 * sizeof(unsigned long long), c->stream));
  hipLaunchKernelGGL(kb, dim3(W), dim3(gpf::STEP_NTH), 0, c->stream, mode, D, Npad, P, L, C, nullptr);
  GPF_HIP(c, hipEventRecord(a, c->stream));
  for (int i = 0; i < iters; ++i)
    hipLaunchKernelGGL(kb, dim3(W), dim3(gpf::STEP_NTH), 0, c->stream, mode, D, Npad, P, L, C, clk);
  GPF_HIP(c, hipEventRecord(b, c->stream));
  GPF_HIP(c, hipEventSynchronize(b));
  c->bench_sclk = read_clock(clk);
  hipFree(clk);
  float ms = 0.f;
  GPF_HIP(c, hipEventElapsedTime(&ms, a, b));
  *tflops = 2.0 * T * T * (double)D * W * iters / (ms * 1e-3) / 1e12;
  hipEventDestroy(a);
  hipEventDestroy(b);
  hipFree(L);
  hipFree(C);
  return GPF_OK;
}

// Debug / measurement hook: the diagonal-block factor (gpf::factor128) on n 128x128 blocks.
int gpf_debug_factor128(gpf_ctx* c, const double* A, const double* y, int n, double* L, double* U, double* z, double* s2,
                        double* sz, int* bad, double* cycles) {
  if (!c || !A || !y || n <= 0 || !L || !U || !z || !s2 || !sz || !bad) return GPF_BAD_ARG;
  hipSetDevice(c->device);
  const size_t nb = (size_t)n * T * T, nv = (size_t)n * T;
  DevBuf dL, dU, dy, ds2, dsz, db, dc;
  GPF_HIP(c, dL.alloc(nb * 8, c->stream));
  GPF_HIP(c, dU.alloc(nb * 8, c->stream));
  GPF_HIP(c, dy.alloc(nv * 8, c->stream));
  GPF_HIP(c, ds2.alloc(nv * 8, c->stream));
  GPF_HIP(c, dsz.alloc(nv * 8, c->stream));
  GPF_HIP(c, db.alloc((size_t)n * 4, c->stream));
  GPF_HIP(c, dc.alloc((size_t)n * 8, c->stream));
  GPF_HIP(c, hipMemcpyAsync(dL.p, A, nb * 8, hipMemcpyHostToDevice, c->stream));
  GPF_HIP(c, hipMemsetAsync(dU.p, 0x7f, nb * 8, c->stream));  // (every entry must be written)
  GPF_HIP(c, hipMemcpyAsync(dy.p, y, nv * 8, hipMemcpyHostToDevice, c->stream));
  GPF_HIP(c, hipMemsetAsync(db.p, 0, (size_t)n * 4, c->stream));
  hipLaunchKernelGGL(gpf::k_debug_factor128, dim3(n), dim3(gpf::DNTH), 0, c->stream, dL.as<double>(), dU.as<double>(),
                     dy.as<double>(), ds2.as<double>(), dsz.as<double>(), db.as<int>(), dc.as<unsigned long long>());
  GPF_HIP(c, hipGetLastError());
  GPF_HIP(c, hipMemcpyAsync(L, dL.p, nb * 8, hipMemcpyDeviceToHost, c->stream));
  GPF_HIP(c, hipMemcpyAsync(U, dU.p, nb * 8, hipMemcpyDeviceToHost, c->stream));
  GPF_HIP(c, hipMemcpyAsync(z, dy.p, nv * 8, hipMemcpyDeviceToHost, c->stream));
  GPF_HIP(c, hipMemcpyAsync(s2, ds2.p, nv * 8, hipMemcpyDeviceToHost, c->stream));
  GPF_HIP(c, hipMemcpyAsync(sz, dsz.p, nv * 8, hipMemcpyDeviceToHost, c->stream));
  GPF_HIP(c, hipMemcpyAsync(bad, db.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
  std::vector<unsigned long long> cyc(n);
  GPF_HIP(c, hipMemcpyAsync(cyc.data(), dc.p, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
  GPF_HIP(c, hipStreamSynchronize(c->stream));
  if (cycles)
    for (int i = 0; i < n; ++i) cycles[i] = (double)cyc[i];
  return GPF_OK;
}

#ifdef GPF_WG_TRACE
// diagnostic builds only: per-workgroup (start, end, placement) of k_step, [J][wg][3]
int gpf_debug_wg_trace(unsigned long long* out, int nj, int nwg) {
  if (!out || nj <= 0 || nwg <= 0 || nj > gpf::WG_TRACE_J || nwg > gpf::WG_TRACE_N) return GPF_BAD_ARG;
  hipDeviceSynchronize();
  std::vector<unsigned long long> h((size_t)gpf::WG_TRACE_J * gpf::WG_TRACE_N * 3);
  if (hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(gpf::g_wg_trace), h.size() * 8) != hipSuccess) return GPF_HIP_ERROR;
  for (int j = 0; j < nj; ++j)
    std::memcpy(out + (size_t)j * nwg * 3, h.data() + (size_t)j * gpf::WG_TRACE_N * 3, (size_t)nwg * 3 * 8);
  return GPF_OK;
}
// diagnostic builds only: wave-0 phase-end stamps of k_step workgroups, [J][wg][4] (see step_item)
int gpf_debug_wg_phase(unsigned long long* out, int nj, int nwg) {
  if (!out || nj <= 0 || nwg <= 0 || nj > gpf::WG_TRACE_J || nwg > gpf::WG_TRACE_N) return GPF_BAD_ARG;
  hipDeviceSynchronize();
  std::vector<unsigned long long> h((size_t)gpf::WG_TRACE_J * gpf::WG_TRACE_N * 4);
  if (hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(gpf::g_wg_phase), h.size() * 8) != hipSuccess) return GPF_HIP_ERROR;
  for (int j = 0; j < nj; ++j)
    std::memcpy(out + (size_t)j * nwg * 4, h.data() + (size_t)j * gpf::WG_TRACE_N * 4, (size_t)nwg * 4 * 8);
  return GPF_OK;
}
#endif


}  // extern "C"

// swarm exchange across ranks (after the C-ABI above: it calls gpf_eval_batch)
#include "gpf_comm.hip"
