// DLAP native engine: device-resident 3-phase GAN training / evaluation for G models at once.
//
// This is the MI355X runtime behind `train_3phase` on a GPU (the reference runs the same
// schedule eagerly on the CPU, `/root/reference/src/train.py:156-426`):
//   * the panel of every split lives in HBM for the whole run, compacted to valid rows
//     (bf16 [R][KP] features + int32 dense index), with dense [T*N] fp32 returns/mask;
//   * G models (ensemble members / sweep configs of one architecture) are batched into the
//     same launches (grid.y = job), so a 9-seed ensemble costs the launches of one model;
//   * an epoch is a fixed launch plan (prologue -> towers -> loss passes -> tower backward ->
//     finalize -> update -> evaluation -> bookkeeping) that reads every step-varying value
//     from device counters, so it is captured ONCE per phase into a hipGraph and replayed;
//   * history, best-epoch tracking and checkpoint snapshots are device-side: the host only
//     synchronises at print intervals / phase boundaries.
#include <cstdint>
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "layout.h"
#include "loss.h"
#include <chrono>
#include "mlp.h"
#include "panel.h"
#include "rnn.h"
#include "update.h"
#include "wide.h"

namespace py = pybind11;

void dlap_throw_hip(hipError_t e, const char* what, const char* file, int line) {
  throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e) + " at " + file + ":" +
                           std::to_string(line) + " (" + what + ")");
}

// Engines of several threads (the sweep runs architecture buckets concurrently) must not issue
// legacy-stream operations (synchronous hipMemcpy / hipMemset / hipMalloc / hipFree) while
// another thread is capturing an epoch graph: every such call and every capture takes this lock.
// Graph replays, the long part of a run, are outside it.
static std::mutex g_legacy_mu;
// Host-blocking HIP calls issued by the engine (synchronous copies / allocations, stream syncs):
// the module-API tests assert that a training step issues none.
static std::atomic<long long> g_blocking{0};
// Engines alive in the process (leak checks in the GPU tests)
static std::atomic<int> g_live_engines{0};
#define HIP_LEGACY(expr)                                \
  do {                                                  \
    std::lock_guard<std::mutex> _legacy_guard(g_legacy_mu); \
    g_blocking.fetch_add(1, std::memory_order_relaxed); \
    HIP_OK(expr);                                       \
  } while (0)

// Retired epoch-graph executors. The runtime completes a graph launch through a handler on
// its own thread that still touches the executor after the launching stream has been
// synchronised; destroying the executor right away and having the allocator hand its memory
// to the next executor crashed the next hipGraphLaunch inside the runtime (measured: the
// pipelined body graph of a fresh engine, created right after the previous engine died, got the
// address of the freshly destroyed one and segfaulted at its first launch). An executor is
// therefore destroyed only when (a) an event recorded on its launch stream at retirement (after
// its last launch) has completed, and (b) at least RETIRE_LAG later executors have been retired
// since (its completion handler long finished). A few hundred stay alive at most (a few KiB each).
struct RetiredExec {
  hipGraphExec_t exec;
  hipEvent_t done;      // recorded after the executor's last launch (nullptr: none recorded)
  long long seq;        // retirement number
};
static std::mutex g_retired_mu;
static std::vector<RetiredExec> g_retired;
static long long g_retire_seq = 0;
static constexpr long long RETIRE_LAG = 256;
static void retire_graph_exec(hipGraphExec_t e, hipStream_t st) {
  hipEvent_t ev = nullptr;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess) {
    if (hipEventRecord(ev, st) != hipSuccess) { (void)hipEventDestroy(ev); ev = nullptr; }
  }
  std::lock_guard<std::mutex> g(g_retired_mu);
  g_retired.push_back({e, ev, g_retire_seq++});
  if (g_retired.size() < 2 * RETIRE_LAG) { (void)hipGetLastError(); return; }
  std::vector<RetiredExec> keep;
  keep.reserve(g_retired.size());
  for (const RetiredExec& r : g_retired) {
    const bool old = g_retire_seq - r.seq >= RETIRE_LAG;
    const bool finished = r.done == nullptr || hipEventQuery(r.done) == hipSuccess;
    if (old && finished) {
      (void)hipGraphExecDestroy(r.exec);
      if (r.done) (void)hipEventDestroy(r.done);
    } else {
      keep.push_back(r);
    }
  }
  g_retired.swap(keep);
  // the statuses above are ignored on purpose (a query of a still-pending event, a destroy the
  // runtime refuses): do not leave one as the thread's sticky error for the next launch check
  (void)hipGetLastError();
}

namespace {

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  void alloc(size_t count, bool zero = true) {
    free();
    n = count;
    if (count == 0) return;
    HIP_LEGACY(hipMalloc(&p, count * sizeof(T)));
    if (zero) HIP_LEGACY(hipMemset(p, 0, count * sizeof(T)));
  }
  void free() {
    if (p) { std::lock_guard<std::mutex> g(g_legacy_mu); (void)hipFree(p); }
    p = nullptr;
    n = 0;
  }
  ~DevBuf() { free(); }
};

struct SplitDev {
  int T = 0, N = 0, R = 0;
  float Nbar = 0.f;
  float Nnorm = 0.f;                 // cross-sectional sharding: the global stock count (0: N)
  DevBuf<uint16_t> X;
  DevBuf<int> rowti, row_ptr;        // rowti: [R] (t, i) int2
  DevBuf<float> Rm, mask, invNt, Nt, meanR, RR, invT, macro, Rc;
  DevBuf<uint16_t> XT;               // wide path, train split: rows-as-k copy of X (k_wgrad0)
  bool set = false;
};

struct ModelSplitWS {   // per (model, split)
  DevBuf<float> pp, abias, xg, xin, sg, sc, sh;
  DevBuf<float> w, wn, h, P, port, sdf, mu, E, Eu, dE, dEu, part, pe, pu, dw, rstat, scal;
  DevBuf<float> u, v, dpp, dab, dg, dx;
  DevBuf<uint32_t> gb;        // SDF dropout keep words of the train split (two parity halves)
  DevBuf<float> scal_prev;    // train split: metrics of the last finished step (bookkeeping)
  DevBuf<float> z;            // wide path: layer-0 pre-activations [ntiles][zc][64][4]
  DevBuf<uint16_t> dzs, dzm;  // wide path, train: layer-0 dz fragments (SDF / moment)
  DevBuf<float> wpart;        // wide path, train: layer-0 weight-gradient partials
  DevBuf<float> h0, c0;       // [nrnn][H] initial LSTM state of the split (zero unless set_hidden)
  DevBuf<float> dh0, dc0;     // train split: dL/d(initial state) from the last LSTM backward
  DevBuf<float> dhx;          // train split, module API: external dL/dh [T*N][K] (lazy)
  DevBuf<double> gram;        // Gram mode: [2][T][T] Gc, Gu of the frozen moments (k_gram.hip)
  DevBuf<double> gpart;       // Gram mode: [T][2] per-period quadratic-form terms
  DevBuf<float> xs;           // sharded engine: [4][T] per-period partial sums + [2] loss sums
};

struct ModelState {
  DevBuf<float> params, grads, m, v, snap_loss, snap_sharpe, gnorm, best, aux, hist, wproj;
  DevBuf<int> adam_step, drop_step, snap_flags, ep, upd_ctr, tail_ctr;
  DevBuf<float> mscr;       // fused backward tail: LSTM step-matrix scratch [T][64]
  DevBuf<uint16_t> blob, blob0;
  unsigned seed = 0;
  unsigned tower_salt = 0;  // XOR-ed (mixed) into the towers' dropout seed only (N-sharding: per rank)
  float lr = 0.f;         // per-model learning rate override (0: use the run's lr)
  float dropout = 0.f;    // per-model dropout rate (sweep members batched in one engine may differ)
};

}  // namespace

// Per-model workgroups of a tower launch over G batched models (grid.y = model): the single-
// model grid tuned at 600x3000 (`one`) divided by G, at least `lo`. The whole launch then keeps
// roughly the single-model workgroup count instead of G times it: fewer weight stagings per
// row and, in the backward, G-fold fewer gradient slabs for k_finalize to reduce. Measured
// (profiles/r3_knobs_grids_batched.log): 9 models 1.045 -> 0.823 ms per epoch, 2 models
// 0.337 -> 0.271 ms.
static int grid_per_model(int one, int lo, int G) { return std::max(lo, one / std::max(1, G)); }

static int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v && *v ? std::atoi(v) : dflt;
}

static void install_crash_handler();
// DLAP_TRACE_HOST=1: one stderr line per host-side engine step (crash localisation on boxes
// where a native backtrace is not available)
static const bool g_htrace = [] { const char* v = std::getenv("DLAP_TRACE_HOST"); return v && *v == '1'; }();
#define HTRACE(...) do { if (g_htrace) { fprintf(stderr, "[dlap-trace] " __VA_ARGS__); fputc('\n', stderr); fflush(stderr); } } while (0)

class Engine {
 public:
  Engine(int F, int M, int nrnn, int H, bool raw_macro_sdf, std::vector<int> hidden,
         std::vector<int> mom_hidden, int K, float dropout, bool normalize_w, bool weighted,
         float residual, int G, int max_epochs, bool fp32)
      : G_(G), max_epochs_(max_epochs) {
    g_live_engines.fetch_add(1);
    HIP_OK(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    {
      // the evaluation stream on a hardware queue of its own: a stream created with a CU mask
      // (here: every CU) gets a dedicated queue instead of one from the runtime's pool, which
      // hands out GPU_MAX_HW_QUEUES (4) queues round robin over all streams of the process. The
      // split epoch graphs wait in-kernel across st_ and st2_; were the two on one queue (a second
      // engine, torch's / RCCL's streams), a wait would sit in front of the work it waits for
      // until it gave up.
      hipDeviceProp_t prop;
      int dev = 0;
      HIP_OK(hipGetDevice(&dev));
      HIP_OK(hipGetDeviceProperties(&prop, dev));
      std::vector<uint32_t> mask((prop.multiProcessorCount + 31) / 32, 0u);
      for (int cu = 0; cu < prop.multiProcessorCount; ++cu) mask[cu / 32] |= 1u << (cu % 32);
      // (measured: no cost against a pooled stream, profiles/r5_eval_queue_ab.log; with a pooled
      // st2_, two live engines deadlocked until the waits gave up)
      HIP_OK(hipExtStreamCreateWithCUMask(&st2_, (uint32_t)mask.size(), mask.data()));
    }
    own_st_ = st_;
    HIP_OK(hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&ev_gram_, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&ev_trgram_, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&ev_mid_, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&ev_a_, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming));
    // evaluation tower grid cap: with the split epoch graphs the evaluation branch has slack and
    // its towers start beside the training chain's loss passes; a narrower grid takes fewer CUs
    // from them -- 224-256 measured best (phase 3 0.1554 vs 0.164 ms at 384, profiles/
    // r5_knobs_eval_gx.log; 384 was best on the round-3 tree). Per job: with G batched models the
    // launch has 2G evaluation jobs, so the per-job grid shrinks with G (see grid_per_model)
    eval_gx_ = env_int("DLAP_EVAL_GX", grid_per_model(256, 64, G));
    zx_eval_ = env_int("DLAP_ZX_EVAL", 1) != 0;
    zx_train_ = env_int("DLAP_ZX_TRAIN", 1) != 0;
    zx_gx_ = std::max(1, env_int("DLAP_ZX_GX", 256));
    h_cache_ = env_int("DLAP_H_CACHE", 1) != 0;
    gram_on_ = env_int("DLAP_GRAM", 1) != 0;
    rnn_overlap_ = env_int("DLAP_RNN_OVERLAP", 1) != 0;
    rnn_overlap_eval_ = env_int("DLAP_RNN_OVERLAP_EVAL", 0) != 0;
    prog_mode_ = env_int("DLAP_PROG_MODE", 1);
    prog_limit_ = (unsigned)env_int("DLAP_PROG_SPIN_LIMIT", 1 << 22);
    fused_p2_ = env_int("DLAP_FUSED_PHASE2", 0) != 0;
    eval_in_fwd_ = env_int("DLAP_EVAL_IN_FWD", 1) != 0;
    eval_sep_ = env_int("DLAP_EVAL_SEP", 0) != 0;
    fused_tail_ = env_int("DLAP_FUSED_TAIL", 1) != 0;
    self_proj_ = env_int("DLAP_SELF_PROJ", 1) != 0;
    tail_adam_ = env_int("DLAP_TAIL_ADAM", 1) != 0;
    tail_adam_pipe_ = env_int("DLAP_TAIL_ADAM", 1) == 2;
    split_graphs_ = env_int("DLAP_SPLIT_GRAPHS", 1) != 0;
    mom_tail_ = env_int("DLAP_MOM_TAIL", 1) != 0;
    train_gram_side_ = env_int("DLAP_TRAIN_GRAM_SIDE", 0) != 0;
    p2_lstm_cache_ = env_int("DLAP_P2_LSTM_CACHE", 1) != 0;
    unroll_ = std::max(1, env_int("DLAP_UNROLL", 8));
    build_desc(F, M, nrnn, H, raw_macro_sdf, hidden, mom_hidden, K, dropout, normalize_w, weighted,
               residual, fp32);
    // fp32 wide path: layer 0 through k_proj0 + the ZIN towers (the fused-layer-0 k_mlp_fwd_zx
    // is bf16 only)
    if (fp32) zx_eval_ = zx_train_ = false;
    prog_.alloc((size_t)G * 3 * 16);      // per (model, split): [0] published periods, [1] spin timeouts
    esync_.alloc(64);                      // split epoch graphs: [0] evaluation recurrences done, [32] consumed
    d_desc_.alloc(sizeof(ModelDesc));
    HIP_LEGACY(hipMemcpy(d_desc_.p, &md_, sizeof(ModelDesc), hipMemcpyHostToDevice));
    models_.resize(G);
    for (int g = 0; g < G; ++g) {
      ModelState& S = models_[g];
      S.dropout = dropout;
      S.params.alloc(md_.P); S.grads.alloc(md_.P); S.m.alloc(md_.P); S.v.alloc(md_.P);
      S.snap_loss.alloc(md_.P); S.snap_sharpe.alloc(md_.P);
      // packed weights: evaluation copy, then the training copy (dropout scale folded in)
      S.gnorm.alloc(1); S.best.alloc(3); S.aux.alloc((size_t)2 * md_.md.aux_floats);
      S.hist.alloc((size_t)max_epochs_ * HIST_W);
      S.adam_step.alloc(2); S.drop_step.alloc(1); S.snap_flags.alloc(2); S.ep.alloc(2); S.upd_ctr.alloc(1);
      S.tail_ctr.alloc(lstm_tail_words());
      S.blob.alloc((size_t)2 * md_.md.blob_frags * 512 * xw());   // bf16 (or fp32: 2 u16 each)
      S.blob0.alloc((size_t)std::max(1, md_.md.b0_frags) * 512 * xw());
      S.wproj.alloc((size_t)(md_.proj_mp + 2) * md_.proj_np);
    }
    ws_.resize((size_t)G * 3);
    build_pack_inverse();
    upload_pack_jobs();
  }
  // Scatter lists of the fused re-pack: pack_index_host names the parameter behind every packed
  // element (from the same gathers k_pack uses), inverted here into
  // fixed-width lists per parameter (PACK_FAN slots). Without them (DLAP_FUSED_PACK=0, indices
  // past fp32's exact integers, or a parameter with more copies) k_pack runs after k_adam.
  void build_pack_inverse() {
    if (env_int("DLAP_FUSED_PACK", 1) == 0 || md_.P >= (1 << 24)) return;
    const int total = pack_total(md_);
    std::vector<int> h(total);
    pack_index_host(md_, h.data());
    std::vector<int> code((size_t)md_.P * PACK_FAN, -1), fan(md_.P, 0);
    for (int e = 0; e < total; ++e) {
      if (h[e] < -1 || h[e] >= md_.P) throw std::runtime_error("pack_index_host: parameter index out of range");
      if (h[e] < 0) continue;
      if (fan[h[e]] == PACK_FAN) return;             // a parameter with more copies: separate k_pack
      code[(size_t)h[e] * PACK_FAN + fan[h[e]]++] = e;
    }
    up(inv_code_, code.data(), code.size());
  }
  // per-model re-pack jobs (buffers allocated in the constructor, never reallocated)
  void upload_pack_jobs() {
    std::vector<UpdJob> pj(G_);
    for (int g = 0; g < G_; ++g) {
      ModelState& S = models_[g];
      pj[g].params = S.params.p;
      pj[g].blob = reinterpret_cast<bf16x8*>(S.blob.p);
      pj[g].blob0 = reinterpret_cast<bf16x8*>(S.blob0.p);
      pj[g].aux = S.aux.p;
      pj[g].wproj = S.wproj.p;
      pj[g].dropout = S.dropout;
    }
    upload(j_pack_, pj);
  }
  ~Engine() {
    g_live_engines.fetch_sub(1);
    HTRACE("~Engine tid=%ld", (long)syscall(SYS_gettid));
    // drain both streams before the graphs, events and (member) buffers go away
    if (st2_) (void)hipStreamSynchronize(st2_);
    if (st_) (void)hipStreamSynchronize(st_);
    if (own_st_ && own_st_ != st_) (void)hipStreamSynchronize(own_st_);
    for (auto& kv : graphs_) retire_graph_exec(kv.second, st_);
    if (ev_fork_) (void)hipEventDestroy(ev_fork_);
    if (ev_join_) (void)hipEventDestroy(ev_join_);
    if (ev_gram_) (void)hipEventDestroy(ev_gram_);
    if (ev_mid_) (void)hipEventDestroy(ev_mid_);
    if (ev_a_) (void)hipEventDestroy(ev_a_);
    for (hipEvent_t e : {ev_in_, ev_out_}) if (e) (void)hipEventDestroy(e);
    if (st2_) (void)hipStreamDestroy(st2_);
    if (own_st_) (void)hipStreamDestroy(own_st_);
    (void)hipGetLastError();      // (ignored statuses above must not fail the next launch check)
  }

  // ---------------------------------------------------------------- description ----------
  py::dict describe() const {
    py::dict d;
    d["P"] = md_.P; d["P_sdf"] = md_.P_sdf; d["KP"] = md_.KP; d["KS1"] = md_.KS1; d["WMB"] = md_.WMB;
    d["Dm"] = md_.Dm; d["blob_frags"] = md_.md.blob_frags; d["aux_floats"] = md_.md.aux_floats;
    d["ntile_s"] = md_.ntile_s; d["tps_s"] = md_.tps_s; d["tbwd"] = md_.tbwd; d["ntile_m"] = md_.ntile_m; d["G"] = G_;
    d["wide"] = md_.md.wide; d["KX"] = md_.md.KX; d["nsplit"] = nsplit_; d["fp32"] = md_.md.fp32;
    return d;
  }

  // ---------------------------------------------------------------- data -----------------
  void set_split(int s, py::array_t<uint16_t, py::array::c_style> X, py::array_t<int, py::array::c_style> rowti,
                 py::array_t<int, py::array::c_style> row_ptr, py::array_t<float, py::array::c_style> Rm,
                 py::array_t<float, py::array::c_style> mask, py::array_t<float, py::array::c_style> macro,
                 int T, int N) {
    const long R = (long)rowti.size() / 2;
    if ((long)X.size() != R * md_.KP * xw())
      throw std::invalid_argument(md_.md.fp32 ? "X must be [R][KP] fp32 (as 2 x uint16)" : "X must be [R][KP] bf16 bits");
    set_split_impl(s, X.data(), false, rowti, row_ptr, Rm, mask, macro, T, N);
  }
  // Same, with the compacted panel X already in device memory (x_ptr: R * KP bf16 values, e.g.
  // a torch CUDA tensor built on the GPU): the scaled panels never round-trip through the host.
  void set_split_dev(int s, uintptr_t x_ptr, long x_elems, py::array_t<int, py::array::c_style> rowti,
                     py::array_t<int, py::array::c_style> row_ptr, py::array_t<float, py::array::c_style> Rm,
                     py::array_t<float, py::array::c_style> mask, py::array_t<float, py::array::c_style> macro,
                     int T, int N) {
    const long R = (long)rowti.size() / 2;
    if (x_elems != R * md_.KP * xw()) throw std::invalid_argument("X must be [R][KP] bf16 (fp32: 2x) elements");
    set_split_impl(s, reinterpret_cast<const uint16_t*>(x_ptr), true, rowti, row_ptr, Rm, mask, macro, T, N);
  }
  void set_split_impl(int s, const uint16_t* Xp, bool x_on_device, py::array_t<int, py::array::c_style> rowti,
                      py::array_t<int, py::array::c_style> row_ptr, py::array_t<float, py::array::c_style> Rm,
                      py::array_t<float, py::array::c_style> mask, py::array_t<float, py::array::c_style> macro,
                      int T, int N) {
    if (s < 0 || s > 2) throw std::invalid_argument("split must be 0, 1 or 2");
    if (T > DLAP_MAX_T) throw std::invalid_argument("T exceeds DLAP_MAX_T");
    SplitDev& D = splits_[s];
    if ((long)rowti.size() / 2 > (long)INT32_MAX) throw std::invalid_argument("too many panel rows");
    const int R = (int)(rowti.size() / 2);
    if ((long)Rm.size() != (long)T * N || (long)mask.size() != (long)T * N) throw std::invalid_argument("Rm/mask must be [T*N]");
    if ((int)row_ptr.size() != T + 1) throw std::invalid_argument("row_ptr must be [T+1]");
    if (md_.M > 0 && (long)macro.size() != (long)T * md_.M) throw std::invalid_argument("macro must be [T][M]");
    D.T = T; D.N = N; D.R = R;
    check_x32(R);
    const size_t nx = (size_t)R * md_.KP * xw();
    if (x_on_device) {
      D.X.alloc(nx, false);
      if (nx) HIP_LEGACY(hipMemcpy(D.X.p, Xp, nx * sizeof(uint16_t), hipMemcpyDeviceToDevice));
    } else {
      up(D.X, Xp, nx);
    }
    up(D.rowti, rowti.data(), (size_t)2 * R);
    {
      std::vector<float> rc(R);
      const int* ti = rowti.data();
      for (int r = 0; r < R; ++r) rc[r] = Rm.data()[(size_t)ti[2 * r] * N + ti[2 * r + 1]];
      up(D.Rc, rc.data(), R);
    }
    up(D.Rm, Rm.data(), (size_t)T * N);
    up(D.mask, mask.data(), (size_t)T * N);
    if (md_.M > 0) up(D.macro, macro.data(), (size_t)T * md_.M);
    // per-period / per-asset constants: the same device kernels as the device-compaction path
    // (set_split_dense), from the uploaded dense Rm / mask, so both paths agree bitwise
    alloc_stats(D, T, N);
    PanelIn in{};
    in.ret = D.Rm.p; in.maskf = D.mask.p; in.T = T; in.N = N;
    PanelOut out = panel_out(D);
    out.dense_out = 0;
    launch_panel_stats(in, out, st_);
    int R_dev = 0;
    finish_stats(D, &R_dev);
    if (R_dev != R) throw std::invalid_argument("mask and compact rows disagree");
    std::vector<int> rp(T + 1);
    HIP_LEGACY(hipMemcpy(rp.data(), D.row_ptr.p, (T + 1) * sizeof(int), hipMemcpyDeviceToHost));
    if (std::memcmp(rp.data(), row_ptr.data(), (T + 1) * sizeof(int)) != 0)
      throw std::invalid_argument("row_ptr does not match the mask");
    finish_split(s);
  }

  // ---- device split preparation (k_panel.hip) ------------------------------------------------
  void alloc_stats(SplitDev& D, int T, int N) {
    D.Nt.alloc(T, false); D.invNt.alloc(T, false); D.meanR.alloc(T, false); D.RR.alloc(T, false);
    D.invT.alloc(std::max(N, 1), false); D.row_ptr.alloc(T + 1, false);
    cnt_scratch_.alloc(std::max(T, 1), false);
    nbar_scratch_.alloc(1, false);
  }
  PanelOut panel_out(SplitDev& D) {
    PanelOut o{};
    o.Rm = D.Rm.p; o.mask = D.mask.p; o.Nt = D.Nt.p; o.invNt = D.invNt.p; o.meanR = D.meanR.p; o.RR = D.RR.p;
    o.invT = D.invT.p; o.cnt = cnt_scratch_.p; o.row_ptr = D.row_ptr.p; o.nbar = nbar_scratch_.p;
    o.KP = md_.KP; o.fp32 = md_.md.fp32; o.dense_out = 1;
    return o;
  }
  // N-bar and the row count to the host (the one synchronisation of a split upload)
  void finish_stats(SplitDev& D, int* R) {
    struct { int r; float nb; } h{};
    HIP_OK(hipMemcpyAsync(&h.r, D.row_ptr.p + D.T, sizeof(int), hipMemcpyDeviceToHost, st_));
    HIP_OK(hipMemcpyAsync(&h.nb, nbar_scratch_.p, sizeof(float), hipMemcpyDeviceToHost, st_));
    sync();
    *R = h.r;
    D.Nbar = h.nb;
  }
  // Dense split already in device memory (torch CUDA tensors: feats [T][N][F] fp32, ret [T][N]
  // fp32, mask [T][N] bool (mask_bool) or fp32 0/1, macro [T][M] fp32 or 0): the compacted
  // layout is built on the GPU -- no host copy of the panel, one synchronisation (the row
  // count). `ext` is the caller's stream the inputs were produced on (joined first); the call
  // returns after the inputs are no longer read.
  void set_split_dense(int s, uintptr_t feats, uintptr_t ret, uintptr_t mask, bool mask_bool, uintptr_t macro,
                       int T, int N, int F, uintptr_t ext) {
    if (s < 0 || s > 2) throw std::invalid_argument("split must be 0, 1 or 2");
    if (T > DLAP_MAX_T) throw std::invalid_argument("T exceeds DLAP_MAX_T");
    if (F != md_.F) throw std::invalid_argument("feature dim does not match the engine");
    if ((long)T * N > (long)INT32_MAX) throw std::invalid_argument("panel too large");
    if (md_.M > 0 && !macro) throw std::invalid_argument("macro series required");
    install_crash_handler();
    join_from(ext);
    SplitDev& D = splits_[s];
    D.T = T; D.N = N;
    D.Rm.alloc((size_t)T * N, false);
    D.mask.alloc((size_t)T * N, false);
    alloc_stats(D, T, N);
    PanelIn in{};
    in.feats = reinterpret_cast<const float*>(feats);
    in.ret = reinterpret_cast<const float*>(ret);
    if (mask_bool) in.maskb = reinterpret_cast<const uint8_t*>(mask);
    else in.maskf = reinterpret_cast<const float*>(mask);
    in.T = T; in.N = N; in.F = F;
    PanelOut out = panel_out(D);
    launch_panel_stats(in, out, st_);
    int R = 0;
    finish_stats(D, &R);
    D.R = R;
    check_x32(R);
    D.rowti.alloc((size_t)2 * std::max(R, 1), false);
    D.Rc.alloc(std::max(R, 1), false);
    D.X.alloc(std::max<size_t>((size_t)R * md_.KP * xw(), 1), false);
    out.rowti = reinterpret_cast<int2*>(D.rowti.p); out.Rc = D.Rc.p; out.X = D.X.p;
    launch_panel_compact(in, out, R, st_);
    if (md_.M > 0) {
      D.macro.alloc((size_t)T * md_.M, false);
      HIP_OK(hipMemcpyAsync(D.macro.p, reinterpret_cast<const void*>(macro), (size_t)T * md_.M * sizeof(float),
                            hipMemcpyDeviceToDevice, st_));
    }
    sync();                                   // the caller may free the inputs on return
    finish_split(s);
  }
  // host copies of a split's compacted layout (tests: the device compaction vs prepare_split)
  py::dict read_split(int s) {
    SplitDev& D = splits_[s];
    sync();
    py::dict d;
    d["T"] = D.T; d["N"] = D.N; d["R"] = D.R; d["Nbar"] = D.Nbar;
    auto dl = [&](auto& buf, size_t n) {
      using E = typename std::remove_reference<decltype(*buf.p)>::type;
      py::array_t<E> a(n);
      if (n) HIP_LEGACY(hipMemcpy(a.mutable_data(), buf.p, n * sizeof(E), hipMemcpyDeviceToHost));
      return a;
    };
    d["X"] = dl(D.X, (size_t)D.R * md_.KP * xw());
    d["rowti"] = dl(D.rowti, (size_t)2 * D.R);
    d["row_ptr"] = dl(D.row_ptr, (size_t)D.T + 1);
    d["Rm"] = dl(D.Rm, (size_t)D.T * D.N); d["mask"] = dl(D.mask, (size_t)D.T * D.N);
    d["Rc"] = dl(D.Rc, (size_t)D.R);
    d["Nt"] = dl(D.Nt, (size_t)D.T); d["invNt"] = dl(D.invNt, (size_t)D.T);
    d["meanR"] = dl(D.meanR, (size_t)D.T); d["RR"] = dl(D.RR, (size_t)D.T); d["invT"] = dl(D.invT, (size_t)D.N);
    d["macro"] = dl(D.macro, (size_t)D.T * md_.M);
    return d;
  }
  void finish_split(int s) {
    SplitDev& D = splits_[s];
    const int R = D.R;
    D.set = true;
    h_valid_ = false;
    alloc_ws(s);
    if (md_.md.wide && s == 0) {    // rows-as-k copy of the train panel for the weight gradient
      const size_t ntl = (size_t)(R + 31) / 32;
      D.XT.alloc(std::max<size_t>(ntl * (md_.md.KX / 16) * 512 * xw(), 1), false);
      if (R > 0) launch_xt_build(D.X.p, D.XT.p, R, md_.md.KX, md_.md.fp32 != 0, st_);
      sync();
    }
    graphs_dirty_ = true;
  }

  // ---------------------------------------------------------------- parameters ----------
  void set_params(int g, py::array_t<float, py::array::c_style> p) {
    check_g(g);
    if ((int)p.size() != md_.P) throw std::invalid_argument("params size mismatch");
    HIP_OK(hipMemcpyAsync(models_[g].params.p, p.data(), md_.P * sizeof(float), hipMemcpyHostToDevice, st_));
    pack(g);
    sync();
    h_valid_ = false;
  }
  py::array_t<float> get_params(int g) { return down(models_[check_g(g)].params); }
  py::array_t<float> get_grads(int g) { return down(models_[check_g(g)].grads); }
  py::array_t<float> get_snapshot(int g, int which) {
    ModelState& S = models_[check_g(g)];
    return down(which == 0 ? S.snap_loss : S.snap_sharpe);
  }
  void load_snapshot(int g, int which) {
    ModelState& S = models_[check_g(g)];
    HIP_OK(hipMemcpyAsync(S.params.p, (which == 0 ? S.snap_loss : S.snap_sharpe).p, md_.P * sizeof(float),
                          hipMemcpyDeviceToDevice, st_));
    pack(g);
    sync();
    h_valid_ = false;
  }
  void set_seed(int g, unsigned seed) { models_[check_g(g)].seed = seed; graphs_dirty_ = true; }
  // salt of the SDF / moment tower dropout stream of model g (0 = none): the LSTM inter-layer
  // masks keep the plain seed, so N-sharded ranks agree on the replicated LSTM while their
  // local stocks draw independent tower masks
  void set_tower_salt(int g, unsigned salt) { models_[check_g(g)].tower_salt = salt; graphs_dirty_ = true; }
  unsigned tower_seed(int g) const {
    const ModelState& S = models_[g];
    return S.tower_salt ? S.seed ^ (S.tower_salt * 0x9E3779B9u + 0x7F4A7C15u) : S.seed;
  }
  void set_lr(int g, float lr) { models_[check_g(g)].lr = lr; graphs_dirty_ = true; }
  // Per-model dropout rate (BASELINE config 4's dropout axis batched inside one engine): the
  // model's keep threshold, its train-blob scale 1/(1-p) and its gradient scale-back all follow
  // it; a batched member with rate p trains bit-identically to a solo engine built with p.
  void set_dropout(int g, float p) {
    check_g(g);
    if (!(p >= 0.f && p < 1.f)) throw std::invalid_argument("dropout must be in [0, 1)");
    models_[g].dropout = p;
    float mx = 0.f;
    for (const ModelState& S : models_) mx = std::max(mx, S.dropout);
    md_.dropout = md_.md.dropout = mx;          // structural switches: any model with dropout
    // (queued graphs and kernels read the descriptor: the synchronous copy must not overtake them)
    sync();
    HIP_LEGACY(hipMemcpy(d_desc_.p, &md_, sizeof(ModelDesc), hipMemcpyHostToDevice));
    upload_pack_jobs();
    pack(g);                                     // its train blob carries the new scale
    h_valid_ = false;
    graphs_dirty_ = true;
  }
  float get_dropout(int g) const { return models_[check_g(g)].dropout; }
  py::dict get_opt_state(int g) {
    ModelState& S = models_[check_g(g)];
    py::dict d;
    d["m"] = down(S.m); d["v"] = down(S.v);
    int hs[2], ds[1];
    HIP_LEGACY(hipMemcpy(hs, S.adam_step.p, sizeof(hs), hipMemcpyDeviceToHost));
    HIP_LEGACY(hipMemcpy(ds, S.drop_step.p, sizeof(ds), hipMemcpyDeviceToHost));
    d["step_sdf"] = hs[0]; d["step_moment"] = hs[1]; d["drop_step"] = ds[0];
    return d;
  }
  void set_opt_state(int g, py::array_t<float, py::array::c_style> m, py::array_t<float, py::array::c_style> v,
                     int step_sdf, int step_mom, int drop_step) {
    ModelState& S = models_[check_g(g)];
    HIP_LEGACY(hipMemcpy(S.m.p, m.data(), md_.P * 4, hipMemcpyHostToDevice));
    HIP_LEGACY(hipMemcpy(S.v.p, v.data(), md_.P * 4, hipMemcpyHostToDevice));
    int hs[2] = {step_sdf, step_mom};
    HIP_LEGACY(hipMemcpy(S.adam_step.p, hs, sizeof(hs), hipMemcpyHostToDevice));
    HIP_LEGACY(hipMemcpy(S.drop_step.p, &drop_step, sizeof(int), hipMemcpyHostToDevice));
  }

  // Bookkeeping state of a model (resume files): epoch counters, per-phase best trackers,
  // snapshot flags, the two best-model snapshots and the history rows written so far.
  py::dict get_tracker_state(int g) {
    ModelState& S = models_[check_g(g)];
    py::dict d;
    int ep[2], fl[2];
    float best[3];
    sync();
    HIP_LEGACY(hipMemcpy(ep, S.ep.p, sizeof(ep), hipMemcpyDeviceToHost));
    HIP_LEGACY(hipMemcpy(fl, S.snap_flags.p, sizeof(fl), hipMemcpyDeviceToHost));
    HIP_LEGACY(hipMemcpy(best, S.best.p, sizeof(best), hipMemcpyDeviceToHost));
    d["epoch"] = ep[0]; d["epoch_in_phase"] = ep[1];
    d["snap_loss_taken"] = fl[0]; d["snap_sharpe_taken"] = fl[1];
    d["best_loss"] = best[0]; d["best_sharpe"] = best[1]; d["best_moment"] = best[2];
    d["snap_loss"] = down(S.snap_loss); d["snap_sharpe"] = down(S.snap_sharpe);
    const int nh = std::min(ep[0], max_epochs_);     // rows past the capacity were not kept
    py::array_t<float> h({nh, (int)HIST_W});
    if (nh) HIP_LEGACY(hipMemcpy(h.mutable_data(), S.hist.p, (size_t)nh * HIST_W * 4, hipMemcpyDeviceToHost));
    d["hist"] = h;
    return d;
  }
  void set_tracker_state(int g, int epoch, int epoch_in_phase, int snap_loss_taken, int snap_sharpe_taken,
                         float best_loss, float best_sharpe, float best_moment,
                         py::array_t<float, py::array::c_style> snap_loss,
                         py::array_t<float, py::array::c_style> snap_sharpe,
                         py::array_t<float, py::array::c_style> hist) {
    ModelState& S = models_[check_g(g)];
    // a record taken past the history capacity holds only the first max_epochs rows (the
    // device drops later rows, get_tracker_state reads min(epoch, max_epochs) of them)
    const int nh = std::min(epoch, max_epochs_);
    if (epoch < 0) throw std::invalid_argument("negative epoch count");
    if (snap_loss.size() != md_.P || snap_sharpe.size() != md_.P) throw std::invalid_argument("snapshot size");
    if (hist.size() != (size_t)nh * HIST_W) throw std::invalid_argument("history size");
    sync();
    int ep[2] = {epoch, epoch_in_phase}, fl[2] = {snap_loss_taken, snap_sharpe_taken};
    float best[3] = {best_loss, best_sharpe, best_moment};
    HIP_LEGACY(hipMemcpy(S.ep.p, ep, sizeof(ep), hipMemcpyHostToDevice));
    HIP_LEGACY(hipMemcpy(S.snap_flags.p, fl, sizeof(fl), hipMemcpyHostToDevice));
    HIP_LEGACY(hipMemcpy(S.best.p, best, sizeof(best), hipMemcpyHostToDevice));
    HIP_LEGACY(hipMemcpy(S.snap_loss.p, snap_loss.data(), md_.P * 4, hipMemcpyHostToDevice));
    HIP_LEGACY(hipMemcpy(S.snap_sharpe.p, snap_sharpe.data(), md_.P * 4, hipMemcpyHostToDevice));
    if (nh) HIP_LEGACY(hipMemcpy(S.hist.p, hist.data(), (size_t)nh * HIST_W * 4, hipMemcpyHostToDevice));
  }

  // ---------------------------------------------------------------- phase control -------
  // Reset the per-phase trackers (reference: fresh best values per phase).
  // Stream-ordered (k_begin_phase after the queued epochs): no host synchronisation.
  void begin_phase(int phase) {
    if (graphs_dirty_) { rebuild_jobs(); graphs_dirty_ = false; }
    const int p = (phase >= 1 && phase <= 3) ? phase : 1;   // any phase's table names the trackers
    launch_begin_phase(as<EpochJob>(j_epoch_[p]), G_, st_);
  }
  py::array_t<int> snap_flags(int g) {
    ModelState& S = models_[check_g(g)];
    sync();
    py::array_t<int> out(2);
    HIP_LEGACY(hipMemcpy(out.mutable_data(), S.snap_flags.p, 2 * sizeof(int), hipMemcpyDeviceToHost));
    return out;
  }
  int epoch_count(int g) {
    sync();
    int ep[2];
    HIP_LEGACY(hipMemcpy(ep, models_[check_g(g)].ep.p, sizeof(ep), hipMemcpyDeviceToHost));
    return ep[0];
  }
  py::array_t<float> history(int g) {
    const int n = std::min(epoch_count(g), max_epochs_);   // rows past the capacity were not kept
    py::array_t<float> out({n, (int)HIST_W});
    if (n) HIP_LEGACY(hipMemcpy(out.mutable_data(), models_[g].hist.p, (size_t)n * HIST_W * 4, hipMemcpyDeviceToHost));
    return out;
  }

  // ---------------------------------------------------------------- execution -----------
  // One epoch of `phase` (1, 2, 3): train step (+ valid/test evaluation in phases 1/3) and
  // the device bookkeeping. `n` epochs are run by replaying the phase graph.
  // Runs n epochs of a phase. With evaluation splits (phases 1 and 3) the epochs are
  // software-pipelined: the evaluation + bookkeeping of epoch e-1 and the forward/backward of
  // epoch e read the same parameters, so they run as two concurrent branches of one hipGraph
  // and join before the Adam update:   head | pipe x (n-1) | tail.
  void run_epochs(int phase, int n, float lr, int ignore_epoch, float sel, bool use_graph) {
    install_crash_handler();
    HTRACE("run_epochs phase=%d n=%d graph=%d dirty=%d", phase, n, (int)use_graph, (int)graphs_dirty_);
    if (!splits_[0].set) throw std::runtime_error("train split not set");
    if (ext_stream_) throw std::runtime_error("run_epochs needs the engine's own streams (set_stream(0, False))");
    if (graphs_dirty_) { rebuild_jobs(); graphs_dirty_ = false; }
    if (n <= 0) return;
    const bool pipe = phase != 2 && n_eval_jobs_ > 0 && pipeline_;
    // the moment net trains in phase 2: the cached moments go stale. Else refresh them (and the
    // Gram matrices); with the pipelined graphs the evaluation splits' Gram builds overlap the
    // head epoch (which trains only) on the evaluation stream
    cur_phase_ = phase;
    if (phase == 2) h_valid_ = false;
    else ensure_moments(true, pipe && use_graph);
    // phase 2: the frozen SDF's LSTM state (no inter-layer dropout) is the same every epoch --
    // computed once here, the epochs project only the moment network's bias table
    if (phase == 2 && p2_lstm_cached()) {
      HTRACE("launch_prologue(phase-2 LSTM, once)");
      launch_prologue(as<RnnJob>(j_rnn_train_), G_, splits_[0].T, dd(), md_, st_, false, true);
      lstm_once_ = true;
    }
    struct OnceScope {
      bool& f;
      ~OnceScope() { f = false; }
    } once_scope{lstm_once_};
    struct GramScope {                    // epoch graphs run the loss in Gram mode
      bool& f;
      explicit GramScope(bool& x) : f(x) { f = true; }
      ~GramScope() { f = false; }
    } gram_scope(gram_run_);
    if (!use_graph || xs_on_) {          // (sharded: the hooks' collectives are enqueued per epoch)
      for (int e = 0; e < n; ++e) enqueue_epoch(phase, lr, ignore_epoch, sel);
      return;
    }
    // One executor per epoch graph. (Measured and dropped in round 4: alternating several
    // executors of the same graph -- every hipGraphLaunch of these multi-branch graphs blocks the
    // host ~one epoch, and the wait is not per executor, profiles/r4_hostgaps_short.txt -- and
    // unrolling several pipelined epochs into one graph: both 2-5% slower.)
    if (!pipe) {
      hipGraphExec_t g = graph_for(graph_key(phase, lr, ignore_epoch, sel, 200 + 10 * (int)lstm_once_ + (int)mom_tail_on(phase)),
                                   [&] { enqueue_epoch(phase, lr, ignore_epoch, sel); });
      for (int e = 0; e < n; ++e) HIP_OK(hipGraphLaunch(g, st_));
      return;
    }
    if (split_graphs(phase)) {
      // the body epochs in graphs of `unroll_` epochs each (the rest one by one): a graph boundary
      // costs ~5-9 us (the last node's system-scope release, the first one's acquire); inside a
      // graph consecutive kernels of one queue follow each other directly
      // (both graphs are captured on the first call, whatever n: the bench's warmup captures
      // what its timed region launches)
      const int nbody = n - 1, ku = unroll_;
      hipGraphExec_t chain = graph_for(graph_key(phase, lr, ignore_epoch, sel, 21),
                                       [&] { enqueue_chain_split(phase, lr); });
      hipGraphExec_t evalg = graph_for(graph_key(phase, lr, ignore_epoch, sel, 22),
                                       [&] { enqueue_eval_split(phase, ignore_epoch, sel); }, st2_);
      hipGraphExec_t chaink = chain, evalk = evalg;
      if (ku > 1) {
        chaink = graph_for(graph_key(phase, lr, ignore_epoch, sel, 1000 + ku),
                           [&] { for (int i = 0; i < ku; ++i) enqueue_chain_split(phase, lr); });
        evalk = graph_for(graph_key(phase, lr, ignore_epoch, sel, 2000 + ku),
                          [&] { for (int i = 0; i < ku; ++i) enqueue_eval_split(phase, ignore_epoch, sel); }, st2_);
      }
      hipGraphExec_t tail = graph_for(graph_key(phase, lr, ignore_epoch, sel, 3),
                                      [&] { enqueue_tail(phase, ignore_epoch, sel); });
      launch_head(phase, lr, ignore_epoch, sel);
      join_eval_gram();
      // the evaluation graphs follow the head on st2_ (its masks / step counters, its weights)
      HIP_OK(hipEventRecord(ev_fork_, st_));
      HIP_OK(hipStreamWaitEvent(st2_, ev_fork_, 0));
      const auto t_l = std::chrono::steady_clock::now();
      int e = 0;
      for (; e + ku <= nbody; e += ku) {
        HIP_OK(hipGraphLaunch(chaink, st_));
        HIP_OK(hipGraphLaunch(evalk, st2_));
      }
      for (; e < nbody; ++e) {
        HIP_OK(hipGraphLaunch(chain, st_));
        HIP_OK(hipGraphLaunch(evalg, st2_));
      }
      host_launch_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t_l).count();
      host_launch_n_ += n - 1;
      // (the last evaluation graph finished before the last chain's update: one event for the
      // stream order the host and later launches rely on)
      HIP_OK(hipEventRecord(ev_join_, st2_));
      HIP_OK(hipStreamWaitEvent(st_, ev_join_, 0));
      HIP_OK(hipGraphLaunch(tail, st_));
      return;
    }
    hipGraphExec_t body = graph_for(graph_key(phase, lr, ignore_epoch, sel, 2),
                                    [&] { enqueue_pipe(phase, lr, ignore_epoch, sel); });
    hipGraphExec_t tail = graph_for(graph_key(phase, lr, ignore_epoch, sel, 3),
                                    [&] { enqueue_tail(phase, ignore_epoch, sel); });
    HTRACE("launch head");
    launch_head(phase, lr, ignore_epoch, sel);
    join_eval_gram();                     // the next graphs evaluate
    const auto t_l = std::chrono::steady_clock::now();
    for (int e = 1; e < n; ++e) HIP_OK(hipGraphLaunch(body, st_));
    host_launch_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t_l).count();
    host_launch_n_ += n - 1;
    HTRACE("launch tail");
    HIP_OK(hipGraphLaunch(tail, st_));
    HTRACE("run_epochs done");
  }
  void set_pipeline(bool on) { pipeline_ = on; }
  // Safe mode (the runner's fallback after a spin wait gave up): no in-kernel
  // wait on work of another launch or queue -- no fused LSTM + tower forward, no split epoch
  // graphs, no Adam in the tail (waits inside one launch on lower-numbered, already dispatched
  // blocks stay). The graphs are rebuilt.
  void set_safe_mode(bool on) {
    safe_mode_ = on;
    rnn_overlap_ = on ? false : env_int("DLAP_RNN_OVERLAP", 1) != 0;
    split_graphs_ = on ? false : env_int("DLAP_SPLIT_GRAPHS", 1) != 0;
    tail_adam_ = on ? false : env_int("DLAP_TAIL_ADAM", 1) != 0;
    // the waits left (inside one launch, on blocks dispatched ahead) get the default patience
    if (on) prog_limit_ = std::max(prog_limit_, 1u << 22);
    graphs_dirty_ = true;
  }
  bool safe_mode_ = false;
  // job tables (and the fused launches' co-residency capacities) current
  void ensure_jobs() { if (graphs_dirty_) { rebuild_jobs(); graphs_dirty_ = false; } }

  // Pieces used by the module-level API / tests (no bookkeeping).
  void forward_split(int s, bool train_mode, bool do_mom, bool wait = true) {
    if (graphs_dirty_) { rebuild_jobs(); graphs_dirty_ = false; }
    fwd_only(s, train_mode, do_mom, wait);
  }
  void train_step(int phase, float lr) {
    if (graphs_dirty_) { rebuild_jobs(); graphs_dirty_ = false; }
    if (phase == 2) h_valid_ = false;
    else ensure_moments();
    enqueue_train(phase, lr);
  }
  void backward_only(int phase, bool wait = true) {   // losses + gradients, no optimiser step
    HTRACE("backward_only phase=%d tid=%ld", phase, (long)syscall(SYS_gettid));
    if (graphs_dirty_) { rebuild_jobs(); graphs_dirty_ = false; }
    if (phase != 2) ensure_moments();
    enqueue_train_grads(phase);
    if (wait) sync();
  }

  // ---- cross-sectional sharding (parallel/xsection.py) ------------------------------------
  // Tower backward of the train split from EXTERNAL loss gradients: the caller evaluates the
  // cross-sectional parts of the loss (sums over all ranks' stocks) itself and hands back
  //   phase 1 / 3: dw   -- dL/d(raw SDF weight) of every compact row [R] (device pointer);
  //   phase 2:     dE   -- dL/dE [N][K] and sdf -- the global SDF_t = 1 + P_t [T].
  // The train forward is recomputed (same dropout step), the loss passes are skipped, and the
  // tower backward + gradient finalisation + LSTM BPTT leave the phase's gradients in `grads`
  // (copy_grads). Stream-ordered on the engine stream, no host synchronisation.
  // dh (phase 2, module API): an external dL/dh [T*N][K] (dense, the moments of the train split)
  // instead of dE / sdf -- a caller's loss of the moments.
  void xs_backward(int phase, uintptr_t dw, uintptr_t dE, uintptr_t sdf, uintptr_t dh = 0) {
    if (graphs_dirty_) { rebuild_jobs(); graphs_dirty_ = false; }
    if (phase < 1 || phase > 3) throw std::invalid_argument("phase must be 1, 2 or 3");
    if (dh) {
      if (phase != 2) throw std::invalid_argument("an external dL/dh needs phase 2 (the moment tower)");
      const SplitDev& D = splits_[0];
      const size_t n = (size_t)D.T * D.N * md_.K;
      if (!j_mlp_bwd_dh_.p) {                     // first use: buffers + job table
        std::vector<MlpJob> mb;
        for (int g = 0; g < G_; ++g) {
          ws(g, 0).dhx.alloc(std::max<size_t>(n, 1), false);
          mb.push_back(mlp_job(g, 0, true, true, true));
          mb.back().dz_out = reinterpret_cast<bf16x8*>(ws(g, 0).dzm.p);
          mb.back().dh_ext = ws(g, 0).dhx.p;
        }
        upload(j_mlp_bwd_dh_, mb);
      }
      for (int g = 0; g < G_; ++g)
        if (n) HIP_OK(hipMemcpyAsync(ws(g, 0).dhx.p, reinterpret_cast<const void*>(dh), n * sizeof(float),
                                     hipMemcpyDeviceToDevice, st_));
    }
    if (phase != 2) ensure_moments();
    const SplitDev& D = splits_[0];
    enqueue_dropmask(phase, 0, st_);
    const bool fused = fused_fwd(phase);
    if (fused) launch_proj(as<RnnJob>(j_rnn_train_), G_, D.T, dd(), md_, st_, train_mom(phase));
    else launch_prologue(as<RnnJob>(j_rnn_train_), G_, D.T, dd(), md_, st_, train_mom(phase));
    const bool zx_train = md_.md.wide && zx_train_;
    if (md_.md.wide && !zx_train)
      launch_proj0(as<WideJob>(j_wide_train_[phase]), G_, gx_proj_[0], md_.md, md_.WMB, st_);
    if (zx_train)
      launch_mlp_fwd_zx(as<MlpJob>(j_mlp_train_[phase]), G_, std::max(1, zx_gx_ / G_), md_.md, md_.WMB, st_, true);
    else if (fused)
      launch_mlp_fwd_rnn(as<MlpJob>(j_mlp_train_[phase]), as<RnnJob>(j_rnn_train_), dd(), G_,
                         fused_train_gx(phase), md_.md, md_.KS1, md_.WMB, md_.H, md_.nrnn, D.T, st_,
                         !train_mom(phase));
    else
      launch_mlp_fwd(as<MlpJob>(j_mlp_train_[phase]), G_, phase == 2 ? gx_fwd_[0] : gx_fwd13_, md_.md, md_.KS1,
                     md_.WMB, st_, !train_mom(phase));
    for (int g = 0; g < G_; ++g) {
      ModelSplitWS& W = ws(g, 0);
      if (phase == 2 && dh) {
        // (the moment tower backward reads dL/dh directly)
      } else if (phase == 2) {
        if (!dE || !sdf) throw std::invalid_argument("phase 2 needs dE and sdf");
        HIP_OK(hipMemcpyAsync(W.dE.p, reinterpret_cast<const void*>(dE), W.dE.n * sizeof(float),
                              hipMemcpyDeviceToDevice, st_));
        HIP_OK(hipMemcpyAsync(W.sdf.p, reinterpret_cast<const void*>(sdf), W.sdf.n * sizeof(float),
                              hipMemcpyDeviceToDevice, st_));
      } else {
        if (!dw) throw std::invalid_argument("phases 1 / 3 need dw");
        if (D.R) HIP_OK(hipMemcpyAsync(W.dw.p, reinterpret_cast<const void*>(dw), (size_t)D.R * sizeof(float),
                                       hipMemcpyDeviceToDevice, st_));
      }
    }
    if (phase == 2)
      launch_mlp_bwd_mom(as<MlpJob>(dh ? j_mlp_bwd_dh_ : j_mlp_bwd_[phase]), G_, gx_bwd_, md_.nslice_m, 1, md_.md,
                         md_.KS1, md_.WMB, slab_stride(), fpw_, st_);
    else
      launch_sdf_bwd(as<MlpJob>(j_mlp_bwd_[phase]));
    if (md_.md.wide)
      launch_wgrad0(as<WideJob>(j_wide_bwd_[phase]), G_, dd(), md_.md, phase == 2, md_.WMB, nsplit_, st_);
    enqueue_train_tail(phase);
  }
  long split_rows(int s) const { return splits_[s].R; }

  // ---- module API (ops/fused.py): stream-ordered, no host synchronisation ----------------
  // Run the engine's launches on an external stream (torch's current stream), so module-level
  // forward / backward calls are ordered with the surrounding torch ops. Epoch graphs need the
  // engine's own streams (run_epochs refuses an external one).
  // (external: run on the stream handle ``st`` -- 0 is the legacy NULL stream, torch's default;
  //  not external: back to the engine's own stream)
  void set_stream(uintptr_t st, bool external) {
    HTRACE("set_stream %p ext=%d tid=%ld", (void*)st, (int)external, (long)syscall(SYS_gettid));
    hipStream_t want = external ? reinterpret_cast<hipStream_t>(st) : own_st_;
    if (want == st_ && external == ext_stream_) return;
    sync();                                   // work queued on the previous stream completes first
    st_ = want;
    ext_stream_ = external;
  }
  // Event handoff with a caller's stream (torch's current stream; 0 = the legacy NULL stream):
  // join_from: the engine's stream waits for the work queued so far on `ext`; join_to: `ext`
  // waits for the work queued so far on the engine's stream. The module API brackets its
  // engine calls with these, so the engine never runs on the caller's (possibly legacy) stream
  // and no host synchronisation is needed.
  void join_from(uintptr_t ext) {
    HIP_OK(hipEventRecord(ev_in_, reinterpret_cast<hipStream_t>(ext)));
    HIP_OK(hipStreamWaitEvent(st_, ev_in_, 0));
  }
  void join_to(uintptr_t ext) {
    HIP_OK(hipEventRecord(ev_out_, st_));
    HIP_OK(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(ext), ev_out_, 0));
  }
  // parameters from device memory (a flat fp32 vector in state_dict order), re-packed in order
  void set_params_dev(int g, uintptr_t src) {
    check_g(g);
    HIP_OK(hipMemcpyAsync(models_[g].params.p, reinterpret_cast<const void*>(src), md_.P * sizeof(float),
                          hipMemcpyDeviceToDevice, st_));
    pack(g, false);
    h_valid_ = false;
  }
  // dropout stream position of model g (module API: fresh masks per forward), no host sync
  void set_drop_step(int g, int step) { launch_set_int(models_[check_g(g)].drop_step.p, step, st_); }
  // device-to-device copies of engine state into caller-owned device memory (stream-ordered)
  long copy_ws(int g, int s, const std::string& name, uintptr_t dst) {
    ModelSplitWS& W = ws(g, s);
    const std::map<std::string, DevBuf<float>*> m = {
        {"wn", &W.wn}, {"h", &W.h}, {"P", &W.P}, {"port", &W.port}, {"scal", &W.scal}, {"pp", &W.pp},
        {"w", &W.w}};
    auto it = m.find(name);
    if (it == m.end()) throw std::invalid_argument("copy_ws: unknown buffer " + name);
    const DevBuf<float>& b = *it->second;
    if (b.n) HIP_OK(hipMemcpyAsync(reinterpret_cast<void*>(dst), b.p, b.n * sizeof(float), hipMemcpyDeviceToDevice, st_));
    return (long)b.n;
  }
  void copy_grads(int g, uintptr_t dst) {
    HIP_OK(hipMemcpyAsync(reinterpret_cast<void*>(dst), models_[check_g(g)].grads.p, md_.P * sizeof(float),
                          hipMemcpyDeviceToDevice, st_));
  }
  // initial LSTM state (h0, c0) [nrnn][H] of split s (device pointers; 0 = back to the zero
  // state). Stream-ordered, no host synchronisation.
  void set_hidden(int g, int s, uintptr_t h, uintptr_t c) {
    ModelSplitWS& W = ws(check_g(g), s);
    const size_t n = (size_t)md_.nrnn * md_.H;
    if (n == 0) return;
    if (h) HIP_OK(hipMemcpyAsync(W.h0.p, reinterpret_cast<const void*>(h), n * 4, hipMemcpyDeviceToDevice, st_));
    else HIP_OK(hipMemsetAsync(W.h0.p, 0, n * 4, st_));
    if (c) HIP_OK(hipMemcpyAsync(W.c0.p, reinterpret_cast<const void*>(c), n * 4, hipMemcpyDeviceToDevice, st_));
    else HIP_OK(hipMemsetAsync(W.c0.p, 0, n * 4, st_));
  }
  // dL/d(h0, c0) [nrnn][H] of the last LSTM backward of the train split (device pointers)
  void copy_hidden_grad(int g, uintptr_t dh, uintptr_t dc) {
    ModelSplitWS& W = ws(check_g(g), 0);
    const size_t n = (size_t)md_.nrnn * md_.H;
    if (n == 0) return;
    HIP_OK(hipMemcpyAsync(reinterpret_cast<void*>(dh), W.dh0.p, n * 4, hipMemcpyDeviceToDevice, st_));
    HIP_OK(hipMemcpyAsync(reinterpret_cast<void*>(dc), W.dc0.p, n * 4, hipMemcpyDeviceToDevice, st_));
  }
  // final LSTM state (h_n, c_n) [nrnn][H] of the train split after a forward: the last step of
  // every layer's saved outputs / cells
  void copy_hidden(int g, uintptr_t dst_h, uintptr_t dst_c) {
    ModelSplitWS& W = ws(check_g(g), 0);
    const int T = splits_[0].T, H = md_.H;
    if (md_.nrnn == 0 || T == 0) return;
    for (int l = 0; l < md_.nrnn; ++l) {
      const size_t off = ((size_t)l * T + (T - 1)) * H;
      HIP_OK(hipMemcpyAsync(reinterpret_cast<float*>(dst_h) + (size_t)l * H, W.sh.p + off, H * sizeof(float),
                            hipMemcpyDeviceToDevice, st_));
      HIP_OK(hipMemcpyAsync(reinterpret_cast<float*>(dst_c) + (size_t)l * H, W.sc.p + off, H * sizeof(float),
                            hipMemcpyDeviceToDevice, st_));
    }
  }

  py::array_t<float> read_ws(int g, int s, const std::string& name) {
    ModelSplitWS& W = ws(g, s);
    const std::map<std::string, DevBuf<float>*> m = {
        {"pp", &W.pp}, {"abias", &W.abias}, {"w", &W.w}, {"wn", &W.wn}, {"mu", &W.mu}, {"h", &W.h}, {"P", &W.P},
        {"port", &W.port}, {"sdf", &W.sdf}, {"E", &W.E}, {"Eu", &W.Eu}, {"dE", &W.dE}, {"dEu", &W.dEu},
        {"dw", &W.dw}, {"scal", &W.scal}, {"u", &W.u}, {"v", &W.v}, {"dpp", &W.dpp}, {"dab", &W.dab},
        {"sg", &W.sg}, {"sc", &W.sc}, {"sh", &W.sh}};
    auto it = m.find(name);
    if (it == m.end()) throw std::invalid_argument("unknown workspace buffer " + name);
    sync();
    return down(*it->second);
  }
  py::array_t<float> read_aux(int g) { sync(); return down(models_[check_g(g)].aux); }
  // Gram matrices [2][T][T] (Gc, Gu) of (model g, split s) as last built (tests)
  py::array_t<double> read_gram(int g, int s) {
    ModelSplitWS& W = ws(check_g(g), s);
    sync();
    py::array_t<double> out(W.gram.n);
    if (W.gram.n) HIP_LEGACY(hipMemcpy(out.mutable_data(), W.gram.p, W.gram.n * sizeof(double), hipMemcpyDeviceToHost));
    return out;
  }
  // (re)build the Gram matrices from the current moments now (tests; run_epochs does it itself)
  void refresh_gram() {
    if (graphs_dirty_) { rebuild_jobs(); graphs_dirty_ = false; }
    cur_phase_ = 0;                          // every split's matrices
    ensure_moments(true);
  }
  bool gram_enabled(int phase) const { return phase == 0 ? gram_eval() : gram_train(phase); }
  // Cost model of the loss mode of one phase: the Gram form saves the dense
  // asset passes every epoch but costs a T x T build per split after each moment refresh; over
  // `epochs` epochs of `phase` use it where epochs x saving > build. A function of the schedule
  // and the shapes only (never of runtime state), so a run split into print segments or resumed
  // mid-phase makes the same choice. Coefficients (us, one model, measured at 600x3000x46 on
  // MI355X, profiles/r3_final_kernel_stats_short.txt, r2_final_kernel_stats.txt): dense asset pass
  // per T N (K+1) element 1.8e-6 (train, one pass) / 6.6e-6 (evaluation, split pass), Gram build
  // per T^2 x inner element 7.7e-8, Gram per-epoch extra per T^2 5e-5. DLAP_GRAM_PLAN=0: Gram
  // wherever it applies (the round-3 behaviour).
  void plan_phase(int phase, int epochs) {
    if (phase < 1 || phase > 3) return;
    plan_tr_[phase] = plan_ev_[phase] = true;
    if (phase == 2 || epochs <= 0 || xs_on_ || env_int("DLAP_GRAM_PLAN", 1) == 0) return;
    // costs in us. The training chain's dense loss (period pass, asset pass, metrics, period
    // backward) over the Gram one: a T N + b T N K (the conditional loss's moment sums), minus
    // the quadratic forms' cq T^2 -- calibrated on the split-graph pipeline at 600x3000x46:
    // Gram saves ~12 us per phase-1 epoch and ~26 us per phase-3 epoch (profiles/
    // r5_knobs_gramplan.log; the round-4 constants made phase 1 dense)
    const double cb = 7.7e-8, cq = 5e-5, cta = 2.07e-5, ctb = 2.43e-6, cde = 6.6e-6;
    const double K = md_.K;
    const SplitDev& D0 = splits_[0];
    if (D0.set && D0.T > 0) {
      const bool cond = phase == 3;
      const double T = D0.T, N = D0.N;
      const double build = cb * T * T * N * (cond ? K : 1.0);
      const double save = cta * T * N + (cond ? ctb * T * N * K : 0.0) - cq * T * T;
      plan_tr_[phase] = epochs * save > build;
    }
    double build = 0.0, save = 0.0;
    for (int sp = 1; sp < 3; ++sp) {
      const SplitDev& D = splits_[sp];
      if (!D.set || D.T == 0) continue;
      const double T = D.T, N = D.N;
      build += cb * T * T * N * K;
      save += cde * T * N * (K + 1.0) - cq * T * T;
    }
    plan_ev_[phase] = epochs * save > build;
    // (A/B of the plan: DLAP_GRAM_PLAN=2 dense evaluation splits, 3 dense train split)
    const int force = env_int("DLAP_GRAM_PLAN", 1);
    if (force == 2) plan_ev_[phase] = false;
    if (force == 3) plan_tr_[phase] = false;
  }
  py::tuple gram_plan(int phase) const {
    const int p = (phase >= 1 && phase <= 3) ? phase : 1;
    return py::make_tuple(plan_tr_[p], plan_ev_[p]);
  }
  py::array_t<uint16_t> read_blob(int g) {
    sync();  // (already synchronous)
    ModelState& S = models_[check_g(g)];
    py::array_t<uint16_t> out(S.blob.n);
    HIP_LEGACY(hipMemcpy(out.mutable_data(), S.blob.p, S.blob.n * 2, hipMemcpyDeviceToHost));
    return out;
  }
  void sync() {
    g_blocking.fetch_add(1, std::memory_order_relaxed);
    join_eval_gram();
    HIP_OK(hipStreamSynchronize(st_));
  }
  uintptr_t stream() const { return (uintptr_t)st_; }

  // ---- cross-sectional sharding on the engine (parallel/xsection.py XSEngine) -------------
  // The engine holds ONE rank's stocks. At every cross-sectional coupling of the epoch it calls
  // `hook(what, which, stream)` (GIL taken; the host is enqueueing, nothing waits) so the caller
  // sums the named rank-local buffers over the ranks, ordered on `stream` (torch.distributed):
  //   "sums1" / "sums2"  per-period sums of the period pass (ws "xs" rows 0 / 1..3) of the splits
  //                      in the bitmask `which` (1: train, 6: valid + test, 1 << s: one split);
  //   "loss"             the dense asset passes' loss sums (ws "xs" [4T, 4T + 2));
  //   "gram"             the Gram matrices (ws "gram", fp64 [2][T][T]) of split mask `which`;
  //   "grads"            (which = phase) the flat gradient vector and the per-period input
  //                      gradients (ws "dpp" [T][Dm], phase 2: "dab" [T][64]) of the train split.
  // Everything else is computed redundantly from the summed values (replicated parameters, LSTM,
  // quadratic forms, Adam). Pipelined / split epoch graphs and the fused tail are off; phases 1
  // and 3 use the Gram-form losses (no per-epoch loss all-reduce at all).
  void set_xs(py::object hook) {
    xs_on_ = !hook.is_none();
    xs_hook_ = hook;
    if (xs_on_) pipeline_ = false;
    fwd_tables_.clear();
    graphs_dirty_ = true;
  }
  // the global per-period constants of split s (device float [T] arrays of the caller, read on
  // the engine stream after join_from): N_t, 1/max(N_t, 1), mean R, sum R^2; Nbar; N (all ranks)
  void xs_set_globals(int s, uintptr_t Nt, uintptr_t invNt, uintptr_t meanR, uintptr_t RR, float Nbar, float Nnorm) {
    SplitDev& D = splits_[s];
    if (!D.set) throw std::runtime_error("split not set");
    const size_t b = (size_t)D.T * sizeof(float);
    HIP_OK(hipMemcpyAsync(D.Nt.p, reinterpret_cast<const void*>(Nt), b, hipMemcpyDeviceToDevice, st_));
    HIP_OK(hipMemcpyAsync(D.invNt.p, reinterpret_cast<const void*>(invNt), b, hipMemcpyDeviceToDevice, st_));
    HIP_OK(hipMemcpyAsync(D.meanR.p, reinterpret_cast<const void*>(meanR), b, hipMemcpyDeviceToDevice, st_));
    HIP_OK(hipMemcpyAsync(D.RR.p, reinterpret_cast<const void*>(RR), b, hipMemcpyDeviceToDevice, st_));
    D.Nbar = Nbar;
    D.Nnorm = Nnorm;
    fwd_tables_.clear();
    graphs_dirty_ = true;
  }
  // device pointer + element count of a workspace buffer (the hook's all-reduce operands)
  py::tuple ws_ptr(int g, int s, const std::string& name) {
    ModelSplitWS& W = ws(check_g(g), s);
    if (name == "xs") return py::make_tuple((uintptr_t)W.xs.p, W.xs.n);
    if (name == "gram") return py::make_tuple((uintptr_t)W.gram.p, W.gram.n);
    if (name == "dpp") return py::make_tuple((uintptr_t)W.dpp.p, W.dpp.n);
    if (name == "dab") return py::make_tuple((uintptr_t)W.dab.p, W.dab.n);
    throw std::invalid_argument("ws_ptr: unknown buffer " + name);
  }
  py::tuple grads_ptr(int g) {
    ModelState& S = models_[check_g(g)];
    return py::make_tuple((uintptr_t)S.grads.p, S.grads.n);
  }

 private:
  int G_, max_epochs_;
  hipStream_t st_ = nullptr;
  hipStream_t own_st_ = nullptr;             // the engine's stream (st_ may be an external one)
  bool ext_stream_ = false;
  DevBuf<char> j_pack_;                      // per-model re-pack jobs
  DevBuf<int> inv_code_;                     // parameter -> packed elements (k_adam's fused re-pack)
  struct FwdTables { DevBuf<char> r, m, l, w; bool built = false; };
  std::map<int, FwdTables> fwd_tables_;      // module-API forward job tables (per split / mode)
  hipStream_t st2_ = nullptr;                // evaluation branch of the pipelined epoch graph
  hipEvent_t ev_fork_ = nullptr, ev_join_ = nullptr, ev_mid_ = nullptr, ev_a_ = nullptr;
  hipEvent_t ev_in_ = nullptr, ev_out_ = nullptr;   // join_from / join_to
  hipEvent_t ev_gram_ = nullptr;                     // deferred evaluation-split Gram builds done
  bool eval_gram_pending_ = false;
  int eval_gx_ = 0;                          // cap on the evaluation tower grid (DLAP_EVAL_GX)
  bool zx_eval_ = true;                      // wide path: fused layer-0 evaluation towers (DLAP_ZX_EVAL)
  bool zx_train_ = true;                     // ... and training forward (DLAP_ZX_TRAIN)
  int zx_gx_ = 256;                          // their workgroups over all evaluation jobs (DLAP_ZX_GX)
                                             // (2: with the evaluation LSTM prologue right behind the training one)
  // Moment cache: the moment net only changes in phase 2, so outside it the moments h of every
  // split are constant (eval mode has no dropout; the train split's only if the moment tower has
  // no dropout-carrying hidden layer). They are computed once (refresh_moments) when the moment
  // parameters may have changed, and the phase-1/3 towers run the SDF tower only.
  bool h_cache_ = true;                      // DLAP_H_CACHE
  bool h_valid_ = false;                     // cached h matches the current moment parameters
  bool cache_train_h() const { return h_cache_ && (md_.nl_m == 1 || md_.dropout == 0.f); }
  // Gram mode (k_gram.hip): while the moments are frozen the losses are quadratic forms in the
  // SDF vector, built once per moment refresh (ensure_moments). Needs the moment cache and, for
  // the conditional form, K % 4 == 0 (16-byte rows of the per-stock moment vectors).
  bool gram_on_ = true;                      // DLAP_GRAM
  bool gram_cond_ok() const { return gram_on_ && h_cache_ && md_.K % 4 == 0; }
  bool gram_train(int phase) const {
    return gram_on_ && h_cache_ && (phase == 1 || (phase == 3 && cache_train_h() && gram_cond_ok()));
  }
  bool gram_eval() const { return gram_cond_ok(); }
  DevBuf<double> gram_scratch_;              // split-K partials of the Gram build
  DevBuf<char> j_gram_[3];                   // Gram build jobs per split (every model)
  DevBuf<char> j_loss_gram_[4];              // phase training loss jobs in Gram mode (epoch graphs)
  bool gram_valid_[3] = {false, false, false};   // G of split s matches the cached moments
  bool gram_run_ = false;                    // inside run_epochs (epoch graphs use Gram mode)
  bool xs_on_ = false;                       // cross-sectional sharding hooks (set_xs)
  py::object xs_hook_;
  void xs_call(const char* what, int which, hipStream_t st) {
    if (!xs_on_) return;
    py::gil_scoped_acquire gil;
    xs_hook_(std::string(what), which, (uintptr_t)st);
  }
  // the period pass, as three launches around the ranks' sums when sharded (loss.h)
  void period_fwd(const LossJob* lj, int njobs, int tmax, hipStream_t st, bool store_wn, int which) {
    if (!xs_on_) { launch_period_fwd(lj, njobs, tmax, st, store_wn); return; }
    launch_period_fwd(lj, njobs, tmax, st, store_wn, 1);
    xs_call("sums1", which, st);
    launch_period_fwd(lj, njobs, tmax, st, store_wn, 2);
    xs_call("sums2", which, st);
    launch_period_fwd(lj, njobs, tmax, st, store_wn, 3);
  }
  // Dense or Gram losses per phase (plan_phase): a Gram build pays off only over enough epochs
  int cur_phase_ = 0;                        // phase of the run being enqueued
  bool plan_tr_[4] = {true, true, true, true}, plan_ev_[4] = {true, true, true, true};
  bool use_gram(int phase) const { return gram_run_ && gram_train(phase) && plan_tr_[phase]; }
  bool eval_gram_now() const { return gram_run_ && gram_eval() && plan_ev_[cur_phase_]; }
  const LossJob* loss_tab(int phase, bool gram) const {
    return gram ? as<LossJob>(j_loss_gram_[phase]) : as<LossJob>(j_loss_train_[phase]);
  }
  // whether the training towers of a phase run the moment network (and so need its
  // per-period bias table from the prologue)
  // fused LSTM + training tower forward (k_mlp_fwd_rnn): the towers trail the recurrence
  // period by period instead of starting after it (DLAP_RNN_OVERLAP=0: two launches)
  double capture_s_ = 0.0;                   // host time spent capturing / instantiating graphs
  bool rnn_overlap_ = true;
  bool rnn_overlap_eval_ = false;            // ... also on the evaluation branch (DLAP_RNN_OVERLAP_EVAL)
  // the evaluation being enqueued runs alone on the GPU (the pipeline's tail, the sequential
  // epoch): fused there in any case -- beside the training chain the spinning tower workgroups
  // of both fused launches compete for the same CUs (profiles/r3_knobs_fused_eval.log)
  bool eval_solo_ = false;
  int prog_mode_ = 1;                        // DLAP_PROG_MODE (see MlpJob::prog_mode)
  unsigned prog_limit_ = 1u << 22;           // DLAP_PROG_SPIN_LIMIT (see MlpJob::prog_limit)
  bool fused_p2_ = false;                    // DLAP_FUSED_PHASE2: fused training forward in phase 2 too
  // pipelined phase-1/3 epochs: the evaluation splits' recurrences run inside the fused training
  // forward (k_mlp_fwd_rnn, ne > 0) and their input projections inside its k_proj launch
  // (one job table: j_rnn_all_ = train jobs, then evaluation jobs); DLAP_EVAL_IN_FWD=0: the
  // evaluation branch runs its own prologue beside the training chain (the round-4 graph)
  bool eval_in_fwd_ = true;
  bool self_proj_ = true;                    // DLAP_SELF_PROJ: recurrences project their own inputs
  DevBuf<char> j_rnn_all_;
  int cap_all_ = 0;                          // co-residency capacity at the longest split's LDS
  DevBuf<int> prog_;
  DevBuf<int> esync_;                        // see split_graphs()
  // Co-residency guarantee of the fused LSTM + tower launches: resident workgroups of the fused
  // kernel on the device (occupancy query, rebuild_jobs) for the train split / the evaluation
  // splits; DLAP_FUSED_CAP overrides (tests of the fallback).
  int cap_train_ = 0, cap_eval_ = 0;
  // grid of a fused launch of njobs jobs wanting `want` tower workgroups each: capped so that
  // (1 + gx) * njobs workgroups are all resident at once; 0 = does not fit (two launches then)
  static int fused_grid(int want, int njobs, int cap) {
    if (cap <= 0 || njobs <= 0) return 0;
    const int gx = std::min(want, cap / njobs - 1);
    return gx >= 16 ? gx : 0;
  }
  int eval_grid() const {
    int gx = std::max(gx_fwd_[1], gx_fwd_[2]);
    if (eval_gx_ > 0) gx = std::min(gx, eval_gx_);
    return gx;
  }
  int train_fwd_grid(int phase) const { return phase == 2 ? gx_fwd_[0] : gx_fwd13_; }
  bool fused_eval() const {
    return rnn_overlap_ && (rnn_overlap_eval_ || eval_solo_ || eval_sep_now_) && md_.nrnn > 0 && !md_.md.wide &&
           n_eval_jobs_ > 0 &&
           mlp_fwd_rnn_supported(md_.md, md_.KS1, md_.WMB, md_.H, md_.nrnn, tmax_eval_) &&
           fused_grid(eval_grid(), n_eval_jobs_, cap_eval_) > 0;
  }
 public:
  double capture_seconds() const { return capture_s_; }
  // phases 1 / 3 only: phase 2's training forward runs on the 1024-workgroup grid, more than the
  // GPU holds at once; that is still deadlock-free (the LSTM workgroup is dispatched first), but
  // with two processes sharing one GPU (the gloo rehearsal) phase-2 epochs stalled until a spin
  // wait gave up (profiles/r3_rehearsal_bench_n2_fused_phase2.log)
  bool fused_fwd(int phase) const {
    if (phase == 2 && !fused_p2_) return false;
    return rnn_overlap_ && md_.nrnn > 0 && !md_.md.wide &&
           mlp_fwd_rnn_supported(md_.md, md_.KS1, md_.WMB, md_.H, md_.nrnn, splits_[0].T) &&
           fused_grid(train_fwd_grid(phase), G_, cap_train_) > 0;
  }
  // the capped grids of the fused launches (valid when fused_fwd / fused_eval)
  int fused_train_gx(int phase) const { return fused_grid(train_fwd_grid(phase), G_, cap_train_); }
  int fused_eval_gx() const { return fused_grid(eval_grid(), n_eval_jobs_, cap_eval_); }
  // evaluation recurrences per model inside the fused training forward, and its grid
  int ne_per_model() const { return G_ > 0 && n_eval_jobs_ % G_ == 0 ? n_eval_jobs_ / G_ : 0; }
  int tmax_fwd_all() const { return std::max(splits_[0].T, tmax_eval_); }
  int fused_all_gx(int phase) const {
    const int ne = ne_per_model();
    if (cap_all_ <= 0 || ne <= 0) return 0;
    const int gx = std::min(train_fwd_grid(phase), cap_all_ / G_ - 1 - ne);
    return gx >= 16 ? gx : 0;
  }
  bool eval_rnn_in_fwd(int phase) const {
    if (!eval_in_fwd_ || phase == 2 || n_eval_jobs_ == 0 || ne_per_model() == 0 || !fused_fwd(phase)) return false;
    if (!mlp_fwd_rnn_supported(md_.md, md_.KS1, md_.WMB, md_.H, md_.nrnn, tmax_fwd_all())) return false;
    return fused_all_gx(phase) > 0;
  }
  // zero the spin-timeout counters (tests: the device poison is permanent otherwise)
  void reset_prog_errors() {
    sync();
    std::vector<int> h((size_t)G_ * 3 * 16);
    HIP_LEGACY(hipMemcpy(h.data(), prog_.p, h.size() * sizeof(int), hipMemcpyDeviceToHost));
    for (int k = 0; k < 3 * G_; ++k) h[16 * k + 1] = 0;
    HIP_LEGACY(hipMemcpy(prog_.p, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice));
    // a wait that gave up leaves its launch's counters behind: rearm them (and Adam's)
    for (ModelState& S : models_) {
      HIP_LEGACY(hipMemset(S.tail_ctr.p, 0, S.tail_ctr.n * sizeof(int)));
      HIP_LEGACY(hipMemset(S.upd_ctr.p, 0, S.upd_ctr.n * sizeof(int)));
    }
    HIP_LEGACY(hipMemset(esync_.p, 0, esync_.n * sizeof(int)));
  }
  py::dict fused_info() const {
    py::dict d;
    d["cap_train"] = cap_train_; d["cap_eval"] = cap_eval_;
    for (int ph = 1; ph <= 3; ++ph) d[("train_gx_p" + std::to_string(ph)).c_str()] = fused_fwd(ph) ? fused_train_gx(ph) : 0;
    d["eval_gx_solo"] = fused_grid(eval_grid(), n_eval_jobs_, cap_eval_);
    // pipelined epochs with the evaluation recurrences inside the fused training forward
    d["cap_all"] = cap_all_;
    d["tail_cap"] = tail_cap_;
    for (int ph = 1; ph <= 3; ph += 2) {
      d[("eval_in_fwd_p" + std::to_string(ph)).c_str()] = eval_rnn_in_fwd(ph);
      d[("all_gx_p" + std::to_string(ph)).c_str()] = eval_rnn_in_fwd(ph) ? fused_all_gx(ph) : 0;
    }
    d["eval_per_model"] = ne_per_model();
    d["fused_tail"] = tail_fused(1);
    d["mom_tail"] = mom_tail_on(2);
    d["p2_lstm_cached"] = p2_lstm_cached();
    d["adam_in_tail"] = adam_in_tail(1) && pipeline_ && eval_rnn_in_fwd(1) && (split_graphs(1) || tail_adam_pipe_);
    d["split_graphs"] = split_graphs(1) && pipeline_;
    d["eval_sep"] = split_graphs(1) && pipeline_ && sep_eval(1);
    d["host_launch_us_per_epoch"] = host_launch_n_ ? 1e6 * host_launch_s_ / host_launch_n_ : 0.0;
    // backward launch shape: fine slabs per model (R-only partition), fine slabs per workgroup
    d["bwd_nfine"] = nfine_; d["bwd_fpw"] = fpw_;
    d["fused_pack"] = inv_code_.p != nullptr;
    d["bwd_lds_fpw1"] = (long)mlp_bwd_lds_bytes(md_.md, slab_stride(), 1);
    d["bwd_lds_fpw4"] = (long)mlp_bwd_lds_bytes(md_.md, slab_stride(), 4);
    return d;
  }
  // spin waits of the fused forward that gave up (0 unless the dispatch-order argument failed)
  int prog_timeouts() {
    sync();
    std::vector<int> h((size_t)G_ * 3 * 16);
    HIP_LEGACY(hipMemcpy(h.data(), prog_.p, h.size() * sizeof(int), hipMemcpyDeviceToHost));
    int n = 0;
    for (int k = 0; k < 3 * G_; ++k) n += h[16 * k + 1];
    return n;
  }
 private:
  bool train_mom(int phase) const { return phase == 2 || (phase == 3 && !cache_train_h()); }
  ModelDesc md_{};
  DevBuf<char> d_desc_;
  SplitDev splits_[3];
  std::vector<ModelState> models_;
  std::vector<ModelSplitWS> ws_;
  DevBuf<float> slab_;
  DevBuf<int> cnt_scratch_;                  // split preparation: per-period counts
  DevBuf<float> nbar_scratch_;               // ... and N-bar
  int nfine_ = 4;                            // fine backward slabs per model and slice (from R)
  int fpw_ = 1;                              // fine slabs per backward workgroup (1 or 4)
  int slabs_stored() const { return nfine_ / fpw_; }
  int gx_bwd_ = 1, gx_fwd_[3] = {1, 1, 1};
  int gx_fwd13_ = 1;                         // training forward grid of phases 1 / 3
  int nsplit_ = 1, gx_proj_[3] = {1, 1, 1};  // wide path: wgrad row splits, proj grid per split
  bool graphs_dirty_ = true;
  std::map<std::string, hipGraphExec_t> graphs_;
  // device job tables
  DevBuf<char> j_rnn_train_, j_rnn_eval_, j_mlp_train_[4], j_mlp_eval_, j_mlp_bwd_[4], j_loss_train_[4],
      j_loss_eval_, j_fin_, j_upd_, j_epoch_[4];
  DevBuf<char> j_wide_train_[4], j_wide_eval_, j_wide_bwd_[4];   // wide path (k_wide.hip)
  DevBuf<char> j_rnn_mom_, j_mlp_mom_, j_wide_mom_;             // moment refresh (every split)
  DevBuf<char> j_mlp_bwd_dh_;                                   // moment backward from an external dL/dh
  DevBuf<char> j_loss_eval_dense_;                              // evaluation loss jobs, dense passes
  int n_mom_jobs_ = 0, tmax_all_ = 0, gx_mom_ = 1;
  int n_mom_tr_ = 0, tmax_mom_tr_ = 0, tmax_mom_ev_ = 0;   // train-split jobs lead the tables
  int n_eval_jobs_ = 0;
  int tmax_eval_ = 0, nmax_eval_ = 0;

  std::string graph_key(int phase, float lr, int ig, float sel, int kind) const {
    char b[160];
    const int p = (phase >= 1 && phase <= 3) ? phase : 0;
    snprintf(b, sizeof b, "%d/%.9g/%d/%.3g/%d/%d%d", phase, lr, ig, sel, kind, (int)plan_tr_[p], (int)plan_ev_[p]);
    return b;
  }
  bool pipeline_ = true;
  // uint16 elements per panel / blob value: 1 (bf16) or 2 (fp32 reference-precision towers)
  long xw() const { return md_.md.fp32 ? 2 : 1; }
  int check_g(int g) const {
    if (g < 0 || g >= G_) throw std::out_of_range("model index");
    return g;
  }
  ModelSplitWS& ws(int g, int s) { return ws_[(size_t)g * 3 + s]; }

  template <typename T>
  void up(DevBuf<T>& b, const T* src, size_t n) {
    b.alloc(n, false);
    if (n) HIP_LEGACY(hipMemcpy(b.p, src, n * sizeof(T), hipMemcpyHostToDevice));
  }
  py::array_t<float> down(const DevBuf<float>& b) {
    sync();
    py::array_t<float> out(b.n);
    if (b.n) HIP_LEGACY(hipMemcpy(out.mutable_data(), b.p, b.n * sizeof(float), hipMemcpyDeviceToHost));
    return out;
  }
  template <typename T>
  DevBuf<char>& upload(DevBuf<char>& b, const std::vector<T>& v) {
    b.alloc(v.size() * sizeof(T), false);
    if (!v.empty()) HIP_LEGACY(hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return b;
  }

  void pack(int g, bool wait = true) {
    launch_pack(nullptr, as<UpdJob>(j_pack_) + g, 1, reinterpret_cast<const ModelDesc*>(d_desc_.p), md_, st_);
    if (wait) sync();
  }

  // ------------------------------------------------------------ model descriptor ------
  void build_desc(int F, int M, int nrnn, int H, bool raw_macro_sdf, const std::vector<int>& hs,
                  const std::vector<int>& hm, int K, float dropout, bool normalize_w, bool weighted,
                  float residual, bool fp32) {
    ModelDesc& d = md_;
    std::memset(&d, 0, sizeof d);
    if (hs.empty() || (int)hs.size() > 4) throw std::invalid_argument("native engine supports 1..4 SDF hidden layers");
    for (int w : hs) if (w < 1 || w > 64) throw std::invalid_argument("SDF hidden widths must be in [1, 64]");
    if ((int)hm.size() > 2) throw std::invalid_argument("native engine supports <= 2 moment hidden layers");
    for (int w : hm) if (w < 1 || w > 64) throw std::invalid_argument("moment hidden widths must be in [1, 64]");
    if (K < 1 || K > 64) throw std::invalid_argument("num_condition_moment must be in [1, 64]");
    if (nrnn > DLAP_MAX_RNN || H > DLAP_MAX_H) throw std::invalid_argument("LSTM too large for the native engine");
    d.F = F; d.M = M; d.nrnn = nrnn; d.H = nrnn > 0 ? H : 0; d.K = K;
    d.Dm = nrnn > 0 ? H : (raw_macro_sdf ? M : 0);
    d.KIN = F + d.Dm;
    // fused path: the per-period inputs are written into the last 8*ceil(Dm/8) columns of the
    // panel row by the tower kernels (k_mlp.hip finish_tile), after the F characteristics
    const int ppw = (d.Dm + 7) / 8 * 8;
    const int ks = (F + ppw + 31) / 32;
    // wide path: layer-0 inputs beyond the 128 columns a fused tower tile holds in registers
    // (or DLAP_WIDE=1) -> layer 0 runs as the streaming k_proj0 / k_wgrad0 GEMMs
    const bool wide = ks > 4 || env_int("DLAP_WIDE", 0) != 0;
    if (wide) {
      d.KS1 = 2;                                    // template slot of the ZIN tower kernels
      d.KSB = 0;                                    // no layer-0 fragments in the tower blob
      d.KP = std::max(32, (F + 31) / 32 * 32);      // panel row = the F characteristics only
    } else {
      d.KS1 = ks <= 2 ? 2 : 4;
      d.KSB = d.KS1;
      d.KP = 32 * d.KS1;
    }
    d.md.ppc = wide ? 0 : d.KP - ppw;
    d.md.ppst = (d.Dm + 3) / 4 * 4;
    d.dropout = dropout; d.normalize_w = normalize_w; d.weighted_loss = weighted; d.residual_factor = residual;
    int off = 0;
    for (int l = 0; l < nrnn; ++l) {
      const int in = l == 0 ? M : H;
      d.lstm_w_ih[l] = off; off += 4 * H * in;
      d.lstm_w_hh[l] = off; off += 4 * H * H;
      d.lstm_b_ih[l] = off; off += 4 * H;
      d.lstm_b_hh[l] = off; off += 4 * H;
    }
    d.nl_s = (int)hs.size();
    for (int j = 0; j < d.nl_s; ++j) {
      const int in = j == 0 ? d.KIN : hs[j - 1];
      PackLayer& L = d.s[j];
      L.w_off = off; L.b_off = off + hs[j] * in; L.out = hs[j]; L.in = in; L.ld = in; L.col0 = 0;
      off += hs[j] * in + hs[j];
    }
    d.so_w = off; off += hs.back();
    d.so_b = off; off += 1;
    d.P_sdf = off;
    std::vector<int> mw(hm);
    mw.push_back(K);
    d.nl_m = (int)mw.size();
    int wmax = 0;
    for (int j = 0; j < d.nl_m; ++j) {
      const int in = j == 0 ? M + F : mw[j - 1];
      PackLayer& L = d.m[j];
      L.w_off = off; L.b_off = off + mw[j] * in; L.out = mw[j];
      L.in = j == 0 ? F : in; L.ld = in; L.col0 = j == 0 ? M : 0;
      off += mw[j] * in + mw[j];
      wmax = std::max(wmax, mw[j]);
    }
    d.P = off;
    d.cm1 = mw[0];
    const int wb = (wmax + 15) / 16;
    d.WMB = wb <= 1 ? 1 : (wb <= 2 ? 2 : 4);
    const int KSM = (d.WMB + 1) / 2;
    MlpDims& D = d.md;
    D.F = F; D.Dm = d.Dm; D.K = K; D.cm1 = d.cm1; D.nrnn = nrnn;
    D.nl_sdf = d.nl_s; D.nl_mom = d.nl_m; D.dropout = dropout;
    D.s_fwd0 = 0; D.s_fwd = 4 * d.KSB; D.s_bwd = D.s_fwd + 8 * (d.nl_s - 1);
    D.m_fwd0 = D.s_bwd + 8 * (d.nl_s - 1); D.m_fwd = D.m_fwd0 + d.WMB * d.KSB;
    D.m_bwd = D.m_fwd + (d.nl_m - 1) * d.WMB * KSM;
    D.s_upp = D.m_bwd + (d.nl_m - 1) * d.WMB * KSM;
    D.ubpp = nrnn > 0 ? (d.Dm + 15) / 16 : 0;
    D.s_wo = D.s_upp + 2 * D.ubpp;
    D.blob_frags = D.s_wo + 2;
    D.a_sb = 0; D.a_wo = 64 * d.nl_s; D.a_bo = D.a_wo + 64; D.a_pp = D.a_bo + 4;
    D.a_mb = D.a_pp + 64 * d.Dm; D.aux_floats = D.a_mb + 64 * d.nl_m;
    D.wide = wide ? 1 : 0;
    D.KX = wide ? d.KP : 0;
    D.KSX = D.KX / 32;
    D.zc = 8 + 2 * d.WMB;
    D.b0_frags = wide ? (4 + d.WMB) * D.KSX : 0;
    D.fp32 = fp32 ? 1 : 0;
    if (fp32 && (size_t)D.blob_frags * 2048 + (size_t)D.aux_floats * 4 > 150 * 1024)
      throw std::invalid_argument("precision fp32: this architecture's fp32 weight fragments exceed the LDS budget");
    if (!fp32 && (size_t)D.b0_frags * 1024 > 160 * 1024)     // (k_mlp_fwd_zx stages them; fp32: L2)
      throw std::invalid_argument("feature dim too large for the wide layer-0 kernel (LDS budget)");
    // gradient tiles: layer-0 chunks first (none on the wide path: k_wgrad0), then one tile per
    // later layer (slice = tile, TPS 1)
    // (wide path: only the per-period input columns W0[:, F:F+Dm] have layer-0 tiles)
    const int C0 = wide ? (d.Dm + 63) / 64 : d.KS1 / 2;
    int t = 0;
    for (int c = 0; c < C0; ++c, ++t)
      d.tile_s[t] = wide ? GradTile{d.s[0].w_off, d.s[0].ld, F, d.s[0].out, d.Dm, c, t, 0, 0}
                         : GradTile{d.s[0].w_off, d.s[0].ld, 0, d.s[0].out, d.KP, c, t, 0, 1};
    for (int j = 1; j < d.nl_s; ++j, ++t)
      d.tile_s[t] = GradTile{d.s[j].w_off, d.s[j].ld, 0, d.s[j].out, d.s[j].in, 0, t, j, 0};
    d.ntile_s = t;
    // one gradient tile per slice (the slices recompute the forward each, but the kernel fits
    // two waves per SIMD: DLAP_BWD1_WPS) measured faster than two tiles sharing one recompute at
    // one wave per SIMD (profiles/r4_bwd_shape.log); DLAP_TPS=2 selects the latter
    const char* tps_env = std::getenv("DLAP_TPS");
    const bool tps2 = (wide || d.KS1 == 2) && d.ntile_s == 2 && tps_env && std::atoi(tps_env) == 2;
    d.tps_s = tps2 ? 2 : 1;
    // the one-pass backward (k_tbwd.hip) where it is instantiated: every gradient tile in one
    // slice, the wide path included (DLAP_TBWD=0: the sliced kernel, kept for the fp32 / wide-row shapes)
    d.tbwd = (env_int("DLAP_TBWD", 1) != 0 && tbwd_supported(D, d.KS1) && d.ntile_s == d.nl_s) ? 1 : 0;
    if (d.tbwd) d.tps_s = d.ntile_s;
    // at least one slice: slice 0 also produces the bias / output / per-period gradients
    d.nslice_s = std::max(1, (d.ntile_s + d.tps_s - 1) / d.tps_s);
    for (int k = 0; k < d.ntile_s; ++k) d.tile_s[k].slice = k / d.tps_s;
    t = 0;
    const int C0m = wide ? 0 : d.KS1 / 2;
    for (int c = 0; c < C0m; ++c, ++t)
      d.tile_m[t] = GradTile{d.m[0].w_off, d.m[0].ld, d.m[0].col0, d.m[0].out, d.m[0].in, c, t, 0, 0};
    for (int j = 1; j < d.nl_m; ++j, ++t)
      d.tile_m[t] = GradTile{d.m[j].w_off, d.m[j].ld, 0, d.m[j].out, d.m[j].in, 0, t, j, 0};
    d.ntile_m = t;
    d.nslice_m = std::max(1, t);
    d.tps_m = 1;
    d.proj_mp = std::max(4, (M + 3) / 4 * 4);
    d.proj_np = ((nrnn > 0 ? 4 * H : 0) + 64 + 15) / 16 * 16;   // whole 16-wide MFMA tiles
    for (int e = 0; e < SLAB_EXTRA; ++e) { d.extra_s[e] = -1; d.extra_m[e] = -1; }
    for (int j = 0; j < d.nl_s; ++j)
      for (int o = 0; o < d.s[j].out; ++o) d.extra_s[j * 64 + o] = d.s[j].b_off + o;
    for (int o = 0; o < hs.back(); ++o) d.extra_s[DLAP_MAXL * 64 + o] = d.so_w + o;
    d.extra_s[DLAP_MAXL * 64 + 64] = d.so_b;
    for (int j = 1; j < d.nl_m; ++j)
      for (int o = 0; o < d.m[j].out; ++o) d.extra_m[j * 64 + o] = d.m[j].b_off + o;
  }

  // the tower tile loops address the compact panel with 32-bit byte offsets (gp32): fused-path
  // panels must stay below 4 GiB (the wide path streams layer 0 through other kernels)
  void check_x32(int R) const {
    if (!md_.md.wide && (size_t)R * md_.KP * xw() * sizeof(uint16_t) >= (size_t(1) << 32) - 256)
      throw std::invalid_argument("compact panel exceeds 4 GiB on the fused layer-0 path");
  }
  int slab_stride() const { return std::max(md_.tps_s, md_.tps_m) * 4096 + SLAB_EXTRA; }
  void launch_sdf_bwd(const MlpJob* jobs) {
    if (md_.tbwd) launch_tbwd_sdf(jobs, G_, gx_bwd_, md_.md, slab_stride(), splits_[0].T, st_);
    else launch_mlp_bwd_sdf(jobs, G_, gx_bwd_, md_.nslice_s, md_.tps_s, md_.md, md_.KS1, slab_stride(), fpw_, st_);
  }

  void alloc_ws(int s) {
    const SplitDev& D = splits_[s];
    const int T = D.T, N = D.N, R = D.R, K = md_.K, H = md_.H;
    for (int g = 0; g < G_; ++g) {
      ModelSplitWS& W = ws(g, s);
      W.pp.alloc((size_t)T * std::max(md_.Dm, 1));
      W.abias.alloc((size_t)T * 64);
      W.xg.alloc((size_t)T * std::max(4 * H, 1));
      W.xin.alloc((size_t)T * std::max(H, 1));
      W.w.alloc((size_t)std::max(R, 1)); W.wn.alloc((size_t)T * N); W.h.alloc((size_t)T * N * K);
      W.P.alloc(T); W.port.alloc(T); W.sdf.alloc(T); W.mu.alloc(T);
      W.E.alloc((size_t)N * K); W.Eu.alloc(N); W.dE.alloc((size_t)N * K); W.dEu.alloc(N);
      W.part.alloc(2 * std::max(((size_t)N * (K + 1) + 255) / 256, ((size_t)N + 15) / 16));
      W.pe.alloc((size_t)DLAP_TCH * N * K); W.pu.alloc((size_t)DLAP_TCH * N);
      W.scal.alloc(SC_NSCAL);
      W.gram.alloc((size_t)2 * T * T); W.gpart.alloc((size_t)2 * std::max(T, 1));
      W.xs.alloc((size_t)4 * T + 8);
      W.h0.alloc((size_t)std::max(md_.nrnn * H, 1)); W.c0.alloc((size_t)std::max(md_.nrnn * H, 1));
      if (s == 0) { W.dh0.alloc((size_t)std::max(md_.nrnn * H, 1)); W.dc0.alloc((size_t)std::max(md_.nrnn * H, 1)); }
      if (s == 0) W.scal_prev.alloc(SC_NSCAL);
      if (md_.residual_factor > 0.f) W.rstat.alloc((size_t)T * 4);
      if (s == 0) {
        W.dw.alloc((size_t)std::max(R, 1));
        W.u.alloc((size_t)R * std::max(md_.Dm, 1));
        W.v.alloc((size_t)R * 64);
        W.dpp.alloc((size_t)T * std::max(md_.Dm, 1));
        W.dab.alloc((size_t)T * 64);
        const size_t ntl = (size_t)(R + 31) / 32;
        W.gb.alloc(std::max<size_t>(2 * ntl * md_.nl_s * 64, 1), false);   // two parity halves
        if (md_.nrnn > 0) {
          W.sg.alloc((size_t)md_.nrnn * T * 4 * H);
          W.sc.alloc((size_t)md_.nrnn * T * H);
          W.sh.alloc((size_t)md_.nrnn * T * H);
          W.dg.alloc((size_t)T * 4 * H);
          W.dx.alloc((size_t)T * H);
        }
      }
    }
    if (s == 0) {
      // backward row partition: nfine_ fine slabs per model (one per workgroup of the tuned
      // single-model grid, 256 at 600x3000), a function of R only -- the gradient summation
      // order is the same whether a model trains alone or batched with others (VERDICT r3
      // item 1). The launch shape (fine slabs per workgroup) is chosen in rebuild_jobs.
      const int ntiles = (R + 31) / 32;
      const int ncoarse = std::max(1, std::min(env_int("DLAP_NSLAB_COARSE", 64), ((ntiles + 3) / 4 + 3) / 4));
      nfine_ = 4 * ncoarse;
      const int nsl = std::max(md_.nslice_s, md_.nslice_m);
      slab_.alloc((size_t)G_ * nsl * nfine_ * slab_stride());
    }
    // tower-forward grids (measured, 600x3000x46 epoch graph): the phase-1/3 training forward
    // runs SDF-only (moments cached) beside the evaluation branch and is fastest with one
    // workgroup per CU (256); phase 2 (moment tower, no evaluation branch) with 1024
    gx_fwd_[s] = std::max(1, std::min(((R + 31) / 32 + 3) / 4,
                                      env_int("DLAP_GX_FWD", G_ <= 2 ? 1024 : grid_per_model(1024, 128, G_))));
    if (s == 0) {
      gx_fwd13_ = std::max(1, std::min(((R + 31) / 32 + 3) / 4, env_int("DLAP_GX_FWD13", grid_per_model(384, 96, G_))));
    }
    if (md_.md.wide) {
      const size_t ntl = (size_t)(R + 31) / 32;
      for (int g = 0; g < G_; ++g) {
        ModelSplitWS& W = ws(g, s);
        W.z.alloc(std::max<size_t>(ntl * md_.md.zc * 256, 1), false);
        if (s == 0) {
          W.dzs.alloc(std::max<size_t>(ntl * 4 * 512 * xw(), 1), false);      // (fp32: 2 u16 each)
          W.dzm.alloc(std::max<size_t>(ntl * md_.WMB * 512 * xw(), 1), false);
        }
      }
      if (s == 0) {
        // split-K of the layer-0 weight gradient: ~8 tiles per workgroup, at most 2 per CU
        nsplit_ = std::max(1, std::min((int)((ntl + 7) / 8), env_int("DLAP_WG_SPLIT", 512)));
        for (int g = 0; g < G_; ++g) ws(g, 0).wpart.alloc(wide_part_floats(md_.md, md_.WMB, nsplit_), false);
      }
      gx_proj_[s] = std::max(1, std::min((int)((ntl + 3) / 4), env_int("DLAP_GX_PROJ", 512)));
    }
    // per-period SDF inputs [T][Dm] are staged in LDS by the tower kernels when small
    int tmax = 0;
    for (int k = 0; k < 3; ++k)
      if (splits_[k].set || k == s) tmax = std::max(tmax, splits_[k].T);
    const int ppf = tmax * md_.md.ppst;
    md_.md.pp_lds_floats = (md_.Dm > 0 && ppf <= 8192 && !env_int("DLAP_PP_GLOBAL", 0)) ? ppf : 0;
  }

  // ------------------------------------------------------------ job tables ------------
  RnnJob rnn_job(int g, int s, bool train, int save = -1) {
    ModelSplitWS& W = ws(g, s);
    SplitDev& D = splits_[s];
    RnnJob J{};
    J.params = models_[g].params.p;
    J.wproj = models_[g].wproj.p;
    J.macro = D.macro.p;
    J.T = D.T;
    J.out = W.pp.p;
    // save: keep the per-layer gates / cells / outputs (BPTT; module API final state);
    // default = train. Only the train split (s == 0) has those buffers.
    if ((save < 0 ? train : save != 0) && md_.nrnn > 0 && s == 0) { J.sg = W.sg.p; J.sc = W.sc.p; J.sh = W.sh.p; }
    J.xg = W.xg.p; J.xin = W.xin.p;
    J.abias = W.abias.p;
    J.step = models_[g].drop_step.p;
    J.h0 = W.h0.p; J.c0 = W.c0.p;
    J.seed = models_[g].seed;
    J.train = train;
    J.dropout = models_[g].dropout;
    if (s == 0 && train) J.prog = prog_ptr(g, 0);
    return J;
  }
  // progress counter of the fused LSTM + tower forward of (model, split); set only on the job
  // tables that launch it (training split: train tables; evaluation splits: the eval tables)
  int* prog_ptr(int g, int s) { return prog_.p + 16 * (3 * g + s); }
  void set_prog(MlpJob& J, int g, int s) {
    J.prog = prog_ptr(g, s); J.prog_err = prog_ptr(g, s) + 1; J.prog_mode = prog_mode_; J.prog_limit = prog_limit_;
  }
  const float* pp_ptr(int g, int s) {
    if (md_.nrnn > 0) return ws(g, s).pp.p;
    if (md_.Dm > 0) return splits_[s].macro.p;   // raw macro feeds the SDF directly
    return nullptr;
  }
  MlpJob mlp_job(int g, int s, bool train, bool do_sdf, bool do_mom) {
    ModelSplitWS& W = ws(g, s);
    SplitDev& D = splits_[s];
    MlpJob J{};
    J.X = reinterpret_cast<const bf16x8*>(D.X.p);
    J.rowti = reinterpret_cast<const int2*>(D.rowti.p);
    J.pp = pp_ptr(g, s);
    J.abias = W.abias.p;
    // train-mode towers read the training copy of the packed weights (k_pack)
    J.blob = reinterpret_cast<const bf16x8*>(models_[g].blob.p + (train ? (size_t)md_.md.blob_frags * 512 * xw() : 0));
    J.blob0 = reinterpret_cast<const bf16x8*>(models_[g].blob0.p);
    J.aux = models_[g].aux.p + (train ? md_.md.aux_floats : 0);
    J.w_out = W.w.p; J.h_out = W.h.p;
    J.dw = W.dw.p; J.dE = W.dE.p; J.Rm = D.Rm.p; J.sdfv = W.sdf.p; J.invT = D.invT.p;
    J.slab = slab_.p;
    J.u_out = W.u.p; J.v_out = W.v.p;
    J.z = reinterpret_cast<const f32x4*>(W.z.p);
    J.step = models_[g].drop_step.p;
    J.R = D.R; J.N = D.N; J.T = D.T;
    J.seed = tower_seed(g);
    J.dropout = models_[g].dropout;
    J.train = train; J.do_sdf = do_sdf; J.do_mom = do_mom;
    if (s == 0 && train) set_prog(J, g, 0);
    const int nsl = std::max(md_.nslice_s, md_.nslice_m);
    J.slab_base = g * nsl * slabs_stored();
    J.nslab = nfine_;
    J.fpw = fpw_;
    return J;
  }
  // wide path: projection (do_sdf / do_mom = towers to project) or weight-gradient job
  // (do_mom = the moment tower's layer 0, else the SDF's)
  WideJob wide_job(int g, int s, bool do_sdf, bool do_mom) {
    ModelSplitWS& W = ws(g, s);
    SplitDev& D = splits_[s];
    WideJob J{};
    J.X = reinterpret_cast<const bf16x8*>(D.X.p);
    J.XT = reinterpret_cast<const bf16x8*>(D.XT.p);
    J.rowti = reinterpret_cast<const int2*>(D.rowti.p);
    J.pp = pp_ptr(g, s);
    J.blob0 = reinterpret_cast<const bf16x8*>(models_[g].blob0.p);
    J.z = reinterpret_cast<f32x4*>(W.z.p);
    J.dz = reinterpret_cast<const bf16x8*>(do_mom ? W.dzm.p : W.dzs.p);
    J.part = W.wpart.p;
    J.grads = models_[g].grads.p;
    J.R = D.R; J.T = D.T;
    J.do_sdf = do_sdf; J.do_mom = do_mom;
    return J;
  }
  LossJob loss_job(int g, int s, int phase, bool gram = false) {
    ModelSplitWS& W = ws(g, s);
    SplitDev& D = splits_[s];
    LossJob J{};
    J.Rm = D.Rm.p; J.mask = D.mask.p; J.invNt = D.invNt.p; J.Nt = D.Nt.p; J.meanR = D.meanR.p;
    J.RR = D.RR.p; J.invT = D.invT.p; J.Nbar = D.Nbar; J.T = D.T; J.N = D.N; J.K = md_.K; J.R = D.R;
    J.row_ptr = D.row_ptr.p; J.rowti = reinterpret_cast<const int2*>(D.rowti.p); J.Rc = D.Rc.p; J.mu = W.mu.p;
    J.normalize = md_.normalize_w; J.weighted = md_.weighted_loss; J.phase = phase;
    J.res_factor = md_.residual_factor;
    J.asset_full = (phase > 0 && asset_full_default()) ? 1 : 0;   // training jobs only
    const float nn = D.Nnorm > 0.f ? D.Nnorm : (float)D.N;   // (sharded: every rank's stocks)
    const float kn = (float)md_.K * nn;
    J.coef_c = phase == 3 ? 2.f / kn : (phase == 2 ? -2.f / kn : 0.f);
    J.coef_u = phase == 1 ? 2.f / nn : 0.f;
    J.Nnorm = nn;
    J.xs = xs_on_ ? W.xs.p : nullptr;
    J.w = W.w.p; J.wn = W.wn.p; J.h = phase == 1 ? nullptr : W.h.p;
    J.P = W.P.p; J.port = phase == 0 ? W.port.p : nullptr; J.sdfv = W.sdf.p;
    J.E = W.E.p; J.Eu = W.Eu.p;
    J.dE = (phase == 2 || phase == 3) ? W.dE.p : nullptr;
    J.dEu = phase == 1 ? W.dEu.p : nullptr;
    J.part = W.part.p; J.pe = W.pe.p; J.pu = W.pu.p; J.dw = W.dw.p; J.rstat = W.rstat.p; J.scal = W.scal.p;
    // the fused forward's progress counter of the (model, split), rearmed by the period pass that
    // follows it (train split; evaluation splits: the fused evaluation forward)
    if ((s == 0 && phase > 0) || s > 0) J.prog_reset = prog_ptr(g, s);
    if (gram) {
      J.gram = 1; J.G = W.gram.p; J.gpart = W.gpart.p;
      J.asset_full = 0;
    }
    return J;
  }
  GramJob gram_job(int g, int s, bool cond) {
    ModelSplitWS& W = ws(g, s);
    SplitDev& D = splits_[s];
    GramJob J{};
    J.h = cond ? W.h.p : nullptr;
    J.Rm = D.Rm.p; J.invT = D.invT.p; J.G = W.gram.p;
    J.T = D.T; J.N = D.N; J.K = md_.K;
    if ((long)D.N * std::max(md_.K, 1) >= (1l << 31) - 16) throw std::runtime_error("gram: N * K exceeds the 32-bit inner index");
    return J;
  }
  // Gram build job tables of every split (rebuild_jobs): the train split's conditional matrix
  // only if its moments are cacheable. One scratch area, reused split after split.
  void build_gram_jobs() {
    // split-K scratch: the train split's region, then one region the valid / test builds share
    // (those two run one after the other, possibly on the evaluation stream beside the train
    // split's build and the first epoch: build_gram(defer))
    const size_t n0 = splits_[0].set ? gram_part_doubles(splits_[0].T, G_) : 0;
    size_t n12 = 0;
    for (int s = 1; s < 3; ++s)
      if (splits_[s].set) n12 = std::max(n12, gram_part_doubles(splits_[s].T, G_));
    gram_scratch_.alloc(std::max<size_t>(n0 + n12, 1), false);
    for (int s = 0; s < 3; ++s) {
      const SplitDev& D = splits_[s];
      if (!D.set || D.T == 0) continue;
      const bool cond = gram_cond_ok() && (s != 0 || cache_train_h());
      const size_t per = (size_t)gram_slices(D.T) * 2 * D.T * D.T;
      double* base = gram_scratch_.p + (s == 0 ? 0 : n0);
      std::vector<GramJob> jobs;
      for (int g = 0; g < G_; ++g) {
        jobs.push_back(gram_job(g, s, cond));
        jobs.back().part = base + per * g;
      }
      upload(j_gram_[s], jobs);
    }
  }
  // Build the Gram matrices of every (model, split) from the current cached moments.
  // Stream-ordered on st_ (no host synchronisation). defer: the evaluation splits' builds go
  // to the evaluation stream st2_ (after the moment refresh queued so far) and
  // eval_gram_pending_ is set: the caller joins ev_gram_ into st_ before the first graph that
  // evaluates (the pipelined head trains only, so they overlap it).
  void build_gram(bool defer = false, int smask = 7) {
    bool forked = false;
    for (int s = 0; s < 3; ++s) {
      if (!((smask >> s) & 1)) continue;
      const SplitDev& D = splits_[s];
      if (!D.set || D.T == 0 || gram_valid_[s]) continue;
      // only what the current run's plan reads (run_epochs sets cur_phase_; 0: everything)
      if (cur_phase_ >= 1 && cur_phase_ <= 3 && !(s == 0 ? plan_tr_[cur_phase_] : plan_ev_[cur_phase_])) continue;
      gram_valid_[s] = true;
      hipStream_t st = st_;
      if ((s > 0 || train_gram_side_) && defer) {
        // the builds read the cached moments: st2_ waits for everything queued on st_ so far --
        // on the wide path the moment refresh itself runs on st_ (ensure_moments), so a build
        // deferred while an earlier one is still pending must fork again, or it reads moments
        // the refresh is still writing (run-to-run differences, profiles/r6_wide_determinism.txt)
        if (!forked) {
          HIP_OK(hipEventRecord(ev_fork_, st_));
          HIP_OK(hipStreamWaitEvent(st2_, ev_fork_, 0));
          forked = true;
        }
        if (s > 0) eval_gram_pending_ = true;
        st = st2_;
      }
      HTRACE("launch_gram split=%d", s);
      launch_gram(as<GramJob>(j_gram_[s]), G_, D.T, gram_slices(D.T), st);
      xs_call("gram", 1 << s, st);         // sharded: G summed over every rank's stocks
      if (s == 0 && st == st2_) {
        HIP_OK(hipEventRecord(ev_trgram_, st2_));
        train_gram_pending_ = true;
      }
    }
    if (eval_gram_pending_) HIP_OK(hipEventRecord(ev_gram_, st2_));
  }
  // st_ waits for the train split's deferred refresh + Gram build (no-op when none is pending)
  void join_train_gram() {
    if (!train_gram_pending_) return;
    HIP_OK(hipStreamWaitEvent(st_, ev_trgram_, 0));
    train_gram_pending_ = false;
  }
  bool train_gram_side_ = false;             // DLAP_TRAIN_GRAM_SIDE
  bool train_gram_pending_ = false;
  hipEvent_t ev_trgram_ = nullptr;
  int tg_part_ = 0;                          // enqueue_train_grads: 1 forward only, 2 the rest
  // The head epoch of a pipelined run. With the train split's moment refresh / Gram build deferred
  // to the evaluation stream, two graphs: the forward (dropout masks, LSTM + towers) overlaps the
  // build, then st_ waits for it and the losses, backward and update follow.
  void launch_head(int phase, float lr, int ig, float sel) {
    if (!train_gram_pending_) {
      hipGraphExec_t head = graph_for(graph_key(phase, lr, ig, sel, 1), [&] { enqueue_head(phase, lr); });
      HIP_OK(hipGraphLaunch(head, st_));
      return;
    }
    hipGraphExec_t a = graph_for(graph_key(phase, lr, ig, sel, 11), [&] {
      tg_part_ = 1;
      enqueue_train_grads(phase);
      tg_part_ = 0;
    });
    hipGraphExec_t b = graph_for(graph_key(phase, lr, ig, sel, 12), [&] {
      tg_part_ = 2;
      enqueue_head(phase, lr);
      tg_part_ = 0;
    });
    HIP_OK(hipGraphLaunch(a, st_));
    join_train_gram();
    HIP_OK(hipGraphLaunch(b, st_));
  }
  // st_ waits for deferred evaluation-split Gram builds (no-op when none is pending)
  void join_eval_gram() {
    if (!eval_gram_pending_) return;
    HIP_OK(hipStreamWaitEvent(st_, ev_gram_, 0));
    eval_gram_pending_ = false;
  }

  void rebuild_jobs() {
    HTRACE("rebuild_jobs");
    // The tail's Adam hand-off derives its launch index from a running arrival count divided by
    // the launch's block count, which depends on the train split: with the device
    // quiescent, rearm the running counts so a new split (or any rebuilt job table) starts them
    // at launch 0 with the bookkeeping signals.
    sync();
    if (st2_) HIP_OK(hipStreamSynchronize(st2_));
    for (ModelState& S : models_) {
      HIP_LEGACY(hipMemset(S.tail_ctr.p, 0, S.tail_ctr.n * sizeof(int)));
      HIP_LEGACY(hipMemset(S.upd_ctr.p, 0, S.upd_ctr.n * sizeof(int)));
    }
    tail_cap_ = splits_[0].set && lstm_tail_supported(md_, splits_[0].T) ? lstm_tail_capacity(md_, splits_[0].T) : 0;
    for (auto& kv : graphs_) retire_graph_exec(kv.second, st_);
    graphs_.clear();
    fwd_tables_.clear();
    j_mlp_bwd_dh_.free();
    {   // backward launch shape over the fixed fine-slab partition: one workgroup per fine slab
        // (the compile-time one-slab kernel). DLAP_BWD_FPW=4 walks four fine slabs per
        // workgroup (weights staged once, fine + coarse LDS images, a quarter of the slabs for
        // k_finalize) if the images fit without losing a workgroup per CU -- measured slower at
        // G = 3 and 9 (the runtime slab loop spills more and every fine slab still pays its
        // reduction: 10.58k vs 10.72k model-epochs/s at G = 9, profiles/r4_bwd_shape.log)
      const int want = env_int("DLAP_BWD_FPW", 1);
      const int tps = std::max(md_.tps_s, md_.tps_m);
      fpw_ = (want == 4 && !md_.tbwd && mlp_bwd_fpw_fits(md_.md, md_.KS1, slab_stride(), tps, 4)) ? 4 : 1;
      gx_bwd_ = nfine_ / fpw_;
    }
    std::vector<RnnJob> rt, re;
    std::vector<LossJob> le, led;
    std::vector<MlpJob> me;
    std::vector<FinJob> fj;
    std::vector<UpdJob> uj;
    std::vector<WideJob> we;
    n_eval_jobs_ = 0; tmax_eval_ = 0; nmax_eval_ = 0;
    for (int g = 0; g < G_; ++g) {
      rt.push_back(rnn_job(g, 0, true));
      for (int s = 1; s < 3; ++s) {
        if (!splits_[s].set) continue;
        re.push_back(rnn_job(g, s, false));
        me.push_back(mlp_job(g, s, false, true, !h_cache_));
        re.back().prog = prog_ptr(g, s);
        set_prog(me.back(), g, s);
        we.push_back(wide_job(g, s, true, !h_cache_));
        le.push_back(loss_job(g, s, 0, gram_eval()));
        led.push_back(loss_job(g, s, 0, false));
        tmax_eval_ = std::max(tmax_eval_, splits_[s].T);
        nmax_eval_ = std::max(nmax_eval_, splits_[s].N);
      }
      ModelSplitWS& W = ws(g, 0);
      FinJob F{};
      const int nsl = std::max(md_.nslice_s, md_.nslice_m);
      F.slab = slab_.p + (size_t)g * nsl * slabs_stored() * slab_stride();
      F.grads = models_[g].grads.p; F.row_ptr = splits_[0].row_ptr.p;
      F.u = W.u.p; F.dpp = W.dpp.p; F.v = W.v.p; F.dab = W.dab.p; F.T = splits_[0].T;
      F.nslab = slabs_stored(); F.group = fpw_ == 1 ? 4 : 1;
      F.dropout = models_[g].dropout;
      fj.push_back(F);
      ModelState& S = models_[g];
      UpdJob U{};
      U.params = S.params.p; U.grads = S.grads.p; U.m = S.m.p; U.v = S.v.p;
      U.adam_step = S.adam_step.p; U.drop_step = S.drop_step.p; U.gnorm = S.gnorm.p;
      U.blob = reinterpret_cast<bf16x8*>(S.blob.p); U.aux = S.aux.p; U.wproj = S.wproj.p;
      U.blob0 = reinterpret_cast<bf16x8*>(S.blob0.p);
      U.dpp = W.dpp.p; U.macro = splits_[0].macro.p; U.sg = W.sg.p; U.sc = W.sc.p; U.sh = W.sh.p;
      U.dg = W.dg.p; U.dx = W.dx.p; U.dab = W.dab.p; U.scal = W.scal.p; U.scal_prev = W.scal_prev.p;
      U.h0 = W.h0.p; U.c0 = W.c0.p; U.dh0 = W.dh0.p; U.dc0 = W.dc0.p;
      U.T = splits_[0].T; U.seed = S.seed; U.lr = S.lr; U.prog = prog_ptr(g, 0); U.dropout = S.dropout;
      U.inv_code = inv_code_.p; U.upd_ctr = S.upd_ctr.p;
      if (splits_[0].set && (S.mscr.n < (size_t)splits_[0].T * 64)) S.mscr.alloc((size_t)std::max(splits_[0].T, 1) * 64, false);
      U.tail_ctr = S.tail_ctr.p; U.mscr = S.mscr.p; U.spin_limit = prog_limit_;
      uj.push_back(U);
    }
    n_eval_jobs_ = (int)le.size();
    {
      std::vector<RnnJob> ra = rt;
      ra.insert(ra.end(), re.begin(), re.end());
      upload(j_rnn_all_, ra);
    }
    {   // co-residency capacity of the fused launches (no GPU query when they cannot run)
      const int force = env_int("DLAP_FUSED_CAP", -1);
      const bool can = rnn_overlap_ && md_.nrnn > 0 && !md_.md.wide;
      cap_train_ = !can || !splits_[0].set ? 0
                   : force >= 0 ? force : mlp_fwd_rnn_capacity(md_.md, md_.KS1, md_.WMB, md_.H, md_.nrnn, splits_[0].T);
      cap_eval_ = !can || n_eval_jobs_ == 0 ? 0
                  : force >= 0 ? force : mlp_fwd_rnn_capacity(md_.md, md_.KS1, md_.WMB, md_.H, md_.nrnn, tmax_eval_);
      cap_all_ = !can || n_eval_jobs_ == 0 || !splits_[0].set ? 0
                 : force >= 0 ? force : mlp_fwd_rnn_capacity(md_.md, md_.KS1, md_.WMB, md_.H, md_.nrnn, tmax_fwd_all());
    }
    if (gram_on_) build_gram_jobs();
    for (bool& v : gram_valid_) v = false;
    upload(j_rnn_train_, rt); upload(j_rnn_eval_, re); upload(j_mlp_eval_, me); upload(j_loss_eval_, le); upload(j_loss_eval_dense_, led);
    upload(j_fin_, fj); upload(j_upd_, uj); upload(j_wide_eval_, we);
    {   // moment refresh: eval-mode moment tower (and its per-period bias) of every split
      std::vector<RnnJob> rm;
      std::vector<MlpJob> mm;
      std::vector<WideJob> wm;
      // the train split's jobs first, then the evaluation splits' (ensure_moments may run the
      // latter on the evaluation stream)
      tmax_all_ = 0; gx_mom_ = 1; n_mom_tr_ = 0; tmax_mom_tr_ = 0; tmax_mom_ev_ = 0;
      for (int grp = 0; grp < 2; ++grp)
        for (int g = 0; g < G_; ++g)
          for (int s = grp ? 1 : 0; s < (grp ? 3 : 1); ++s) {
            if (!splits_[s].set) continue;
            rm.push_back(rnn_job(g, s, false));
            mm.push_back(mlp_job(g, s, false, false, true));
            wm.push_back(wide_job(g, s, false, true));
            tmax_all_ = std::max(tmax_all_, splits_[s].T);
            (grp ? tmax_mom_ev_ : tmax_mom_tr_) = std::max(grp ? tmax_mom_ev_ : tmax_mom_tr_, splits_[s].T);
            gx_mom_ = std::max(gx_mom_, gx_fwd_[s]);
            if (!grp) ++n_mom_tr_;
          }
      n_mom_jobs_ = (int)mm.size();
      upload(j_rnn_mom_, rm); upload(j_mlp_mom_, mm); upload(j_wide_mom_, wm);
    }
    for (int phase = 1; phase <= 3; ++phase) {
      std::vector<MlpJob> mt, mb;
      std::vector<LossJob> lt, lg;
      std::vector<EpochJob> ej;
      std::vector<WideJob> wt, wb;
      for (int g = 0; g < G_; ++g) {
        mt.push_back(mlp_job(g, 0, true, true, train_mom(phase)));
        mb.push_back(mlp_job(g, 0, true, true, true));
        mb.back().dz_out = reinterpret_cast<bf16x8*>(phase == 2 ? ws(g, 0).dzm.p : ws(g, 0).dzs.p);
        mt.back().z_out = reinterpret_cast<f32x4*>(ws(g, 0).z.p);
        mt.back().store_mz = phase == 2;
        wt.push_back(wide_job(g, 0, true, train_mom(phase)));
        wb.push_back(wide_job(g, 0, phase != 2, phase == 2));
        // the SDF keep words of the step (k_dropmask), read by its forward and backward
        if (phase != 2) {
          mt.back().gbits = mb.back().gbits = ws(g, 0).gb.p;
          mt.back().gb_half = mb.back().gb_half = ((splits_[0].R + 31) / 32) * md_.nl_s * 64;
        }
        lt.push_back(loss_job(g, 0, phase));
        lg.push_back(loss_job(g, 0, phase, gram_train(phase)));
        ModelState& S = models_[g];
        EpochJob E{};
        E.sc_train = ws(g, 0).scal_prev.p;
        E.sc_valid = (phase != 2 && splits_[1].set) ? ws(g, 1).scal.p : nullptr;
        E.sc_test = (phase != 2 && splits_[2].set) ? ws(g, 2).scal.p : nullptr;
        E.gnorm = S.gnorm.p; E.hist = S.hist.p; E.ep = S.ep.p; E.best = S.best.p;
        E.snap_flags = S.snap_flags.p; E.params = S.params.p;
        E.snap_loss = S.snap_loss.p; E.snap_sharpe = S.snap_sharpe.p;
        E.max_ep = max_epochs_;
        E.prog = prog_ptr(g, 0);
        E.eval_gen = S.tail_ctr.p + TAIL_EVGEN;
        ej.push_back(E);
      }
      upload(j_mlp_train_[phase], mt); upload(j_mlp_bwd_[phase], mb); upload(j_loss_train_[phase], lt);
      upload(j_loss_gram_[phase], lg);
      upload(j_epoch_[phase], ej); upload(j_wide_train_[phase], wt); upload(j_wide_bwd_[phase], wb);
    }
    // evaluation-only jobs of the train split (module API / final evaluation)
    {
      std::vector<MlpJob> mt;
      std::vector<LossJob> lt;
      std::vector<WideJob> wt;
      for (int g = 0; g < G_; ++g) {
        mt.push_back(mlp_job(g, 0, false, true, true));
        lt.push_back(loss_job(g, 0, 0));
        wt.push_back(wide_job(g, 0, true, true));
      }
      upload(j_mlp_train_[0], mt);
      upload(j_loss_train_[0], lt);
      upload(j_wide_train_[0], wt);
    }
  }

  const ModelDesc* dd() const { return reinterpret_cast<const ModelDesc*>(d_desc_.p); }
  template <typename T>
  static const T* as(const DevBuf<char>& b) { return reinterpret_cast<const T*>(b.p); }

  // Recompute the cached moments of every split (enqueued on st_, ahead of the epochs that
  // read them) if the moment parameters may have changed since they were computed.
  // with_gram: also (re)build the Gram matrices (epoch graphs: run_epochs); the module-API
  // steps use the dense loss passes and skip it.
  void ensure_moments(bool with_gram = false, bool defer_eval_gram = false) {
    if (!h_cache_ || n_mom_jobs_ == 0) return;
    if (h_valid_) {
      if (with_gram && gram_on_) build_gram(defer_eval_gram);
      return;
    }
    HTRACE("ensure_moments jobs=%d tmax=%d gx=%d", n_mom_jobs_, tmax_all_, gx_mom_);
    const int n_ev = n_mom_jobs_ - n_mom_tr_;
    if (defer_eval_gram && gram_on_ && !md_.md.wide && n_mom_tr_ > 0 && n_ev > 0) {
      // the evaluation splits' moments (and then their Gram builds, build_gram) on the
      // evaluation stream: only the train split's refresh + Gram precede the head epoch (which
      // trains only); the first graph that evaluates joins them (join_eval_gram)
      HIP_OK(hipEventRecord(ev_fork_, st_));
      HIP_OK(hipStreamWaitEvent(st2_, ev_fork_, 0));
      eval_gram_pending_ = true;
      HTRACE("launch_prologue (moments, split)");
      // (train_gram_side_: the train split's refresh and Gram build too, ahead of the evaluation
      // splits' -- the head epoch's forward needs neither, its loss pass waits, launch_head)
      hipStream_t sm = train_gram_side_ ? st2_ : st_;
      launch_prologue(as<RnnJob>(j_rnn_mom_), n_mom_tr_, tmax_mom_tr_, dd(), md_, sm, true, false);
      launch_mlp_fwd(as<MlpJob>(j_mlp_mom_), n_mom_tr_, gx_mom_, md_.md, md_.KS1, md_.WMB, sm);
      for (bool& v : gram_valid_) v = false;
      if (train_gram_side_) build_gram(true, 1);          // (the head's loss pass waits for it first)
      launch_prologue(as<RnnJob>(j_rnn_mom_) + n_mom_tr_, n_ev, tmax_mom_ev_, dd(), md_, st2_, true, false);
      launch_mlp_fwd(as<MlpJob>(j_mlp_mom_) + n_mom_tr_, n_ev, gx_mom_, md_.md, md_.KS1, md_.WMB, st2_);
      h_valid_ = true;
      build_gram(true);
      return;
    }
    HTRACE("launch_prologue");
    launch_prologue(as<RnnJob>(j_rnn_mom_), n_mom_jobs_, tmax_all_, dd(), md_, st_, true, false);
    if (md_.md.wide && zx_eval_) {
      HTRACE("launch_mlp_fwd_zx");
      launch_mlp_fwd_zx(as<MlpJob>(j_mlp_mom_), n_mom_jobs_, std::max(1, zx_gx_ / n_mom_jobs_), md_.md, md_.WMB, st_);
    } else {
      if (md_.md.wide) launch_proj0(as<WideJob>(j_wide_mom_), n_mom_jobs_, std::max({gx_proj_[0], gx_proj_[1], gx_proj_[2]}),
                                    md_.md, md_.WMB, st_);
      HTRACE("launch_mlp_fwd");
      launch_mlp_fwd(as<MlpJob>(j_mlp_mom_), n_mom_jobs_, gx_mom_, md_.md, md_.KS1, md_.WMB, st_);
    }
    h_valid_ = true;
    for (bool& v : gram_valid_) v = false;
    if (with_gram && gram_on_) build_gram(defer_eval_gram);
  }
  bool dropmask_on(int phase) const { return md_.dropout > 0.f && phase != 2; }
  // keep masks of the step *drop_step + offset* (phases 1/3: the SDF tower's dropout)
  void enqueue_dropmask(int phase, int offset, hipStream_t st) {
    if (!dropmask_on(phase)) return;
    HTRACE("launch_dropmask");
    launch_dropmask(as<MlpJob>(j_mlp_train_[phase]), G_, (splits_[0].R + 31) / 32, md_.md, offset, st);
  }
  // premasked: this step's keep masks were generated by the previous epoch graph.
  // mark: record ev_a_ after the tower forward (2);
  // defer_metrics: the train split's metrics are left to the caller (it records ev_mid_ after the
  // asset pass; the pipelined epoch runs them on the evaluation branch, off the critical chain).
  // eval_rnn: the evaluation splits' projections and recurrences ride in the training prologue
  // and fused forward (eval_rnn_in_fwd; the caller's evaluation branch starts at its towers)
  void enqueue_train_grads(int phase, bool premasked = false, int mark = 0, bool defer_metrics = false,
                           bool eval_rnn = false) {
    const SplitDev& D = splits_[0];
    const bool gram = use_gram(phase);
    const LossJob* lj = loss_tab(phase, gram);
    // (tg_part_: the head epoch split around the wait for a deferred train Gram build, launch_head)
    if (tg_part_ != 2) {
    if (!premasked) enqueue_dropmask(phase, 0, st_);
    // the latency-bound LSTM first, before the streaming projection loads the memory system
    // (fused: only its input projection here, the recurrence runs inside the tower launch)
    const bool fused = fused_fwd(phase);
    // the recurrences project their own inputs inside the fused launch unless the towers need the
    // moment network's per-period bias table (k_proj's other output)
    const bool selfproj = fused && self_proj_ && !train_mom(phase) && !md_.md.wide;
    HTRACE("launch_prologue fused=%d eval_rnn=%d selfproj=%d", (int)fused, (int)eval_rnn, (int)selfproj);
    if (selfproj) {}
    else if (eval_rnn) launch_proj(as<RnnJob>(j_rnn_all_), G_ + n_eval_jobs_, tmax_fwd_all(), dd(), md_, st_, train_mom(phase));
    else if (fused) launch_proj(as<RnnJob>(j_rnn_train_), G_, D.T, dd(), md_, st_, train_mom(phase));
    else if (phase == 2 && lstm_once_) launch_prologue(as<RnnJob>(j_rnn_train_), G_, D.T, dd(), md_, st_, true, false);
    else launch_prologue(as<RnnJob>(j_rnn_train_), G_, D.T, dd(), md_, st_, train_mom(phase));
    // pipelined epoch, train_first_ == 2: the evaluation branch's LSTM prologue is enqueued right
    // behind the training one, so its (serial, few-CU) recurrence starts at the epoch start
    // instead of behind every training-chain node of the graph
    if (eval_prologue_hook_) { enqueue_eval_prologue(eval_prologue_hook_); eval_prologue_hook_ = nullptr; }
    const bool zx_train = md_.md.wide && zx_train_;
    if (md_.md.wide && !zx_train)
      launch_proj0(as<WideJob>(j_wide_train_[phase]), G_, gx_proj_[0], md_.md, md_.WMB, st_);
    if (zx_train)      // layer 0 streamed inside the training towers, z stored for the backward
      launch_mlp_fwd_zx(as<MlpJob>(j_mlp_train_[phase]), G_, std::max(1, zx_gx_ / G_), md_.md, md_.WMB, st_, true);
    else if (eval_rnn)
      launch_mlp_fwd_rnn(as<MlpJob>(j_mlp_train_[phase]), as<RnnJob>(j_rnn_all_), dd(), G_, fused_all_gx(phase),
                         md_.md, md_.KS1, md_.WMB, md_.H, md_.nrnn, tmax_fwd_all(), st_, !train_mom(phase),
                         ne_per_model(), selfproj, fwd_esig_);
    else if (fused)
      launch_mlp_fwd_rnn(as<MlpJob>(j_mlp_train_[phase]), as<RnnJob>(j_rnn_train_), dd(), G_,
                         fused_train_gx(phase), md_.md, md_.KS1, md_.WMB, md_.H, md_.nrnn, D.T, st_,
                         !train_mom(phase), 0, selfproj);
    else
      launch_mlp_fwd(as<MlpJob>(j_mlp_train_[phase]), G_, phase == 2 ? gx_fwd_[0] : gx_fwd13_, md_.md, md_.KS1,
                     md_.WMB, st_, !train_mom(phase));
    if (mark == 2) HIP_OK(hipEventRecord(ev_a_, st_));
    }
    if (tg_part_ == 1) return;
    HTRACE("launch_period_fwd");
    period_fwd(lj, G_, D.T, st_, false, 1);
    if (!gram) {
      if (xs_on_ && phase != 2)
        throw std::runtime_error("sharded engine: phases 1 / 3 need the Gram-form losses (K % 4 == 0, cached moments)");
      HTRACE("launch_asset");
      launch_asset(lj, G_, D.N, md_.K, st_, asset_full_default());
      if (xs_on_) { launch_xs_loss_sums(lj, G_, st_); xs_call("loss", 1, st_); }
    } else {
      // Gram mode: the quadratic-form loss terms and dL/dw come from one per-period pass, which
      // the job metrics (the loss values) then read
      HTRACE("launch_period_bwd(gram)");
      launch_period_bwd(lj, G_, D.T, st_);
    }
    if ((tail_metrics_ && phase != 2) || mom_tail(phase)) {
      // the train split's metrics are computed by the backward tail (enqueue_train_tail)
    } else if (defer_metrics && phase != 2) {
      HIP_OK(hipEventRecord(ev_mid_, st_));
    } else {
      // (k_job_metrics, not the metrics workgroup of k_period_bwd<true>: the same reduction
      // order as the deferred launch of the pipelined epochs, so both schedules are bitwise equal)
      HTRACE("launch_job_metrics");
      launch_job_metrics(lj, G_, st_);
    }
    if (phase == 2) {
      HTRACE("launch_mlp_bwd_mom");
      launch_mlp_bwd_mom(as<MlpJob>(j_mlp_bwd_[phase]), G_, gx_bwd_, md_.nslice_m, 1, md_.md, md_.KS1,
                         md_.WMB, slab_stride(), fpw_, st_);
    } else {
      if (!gram) {
        HTRACE("launch_period_bwd");
        launch_period_bwd(lj, G_, D.T, st_);
      }
      HTRACE("launch_mlp_bwd_sdf");
      launch_sdf_bwd(as<MlpJob>(j_mlp_bwd_[phase]));
    }
    if (md_.md.wide)   // layer-0 weight gradient from the tower's dz fragments
      launch_wgrad0(as<WideJob>(j_wide_bwd_[phase]), G_, dd(), md_.md, phase == 2, md_.WMB, nsplit_, st_);
    enqueue_train_tail(phase);
  }
  // k_finalize -> k_lstm_bwd -> k_wgrad as one launch (k_lstm_tail) where it applies
  bool fused_tail_ = true;                   // DLAP_FUSED_TAIL
  // the pipelined eval-in-forward epoch: the train split's job metrics run in the backward tail
  // (one more block of k_lstm_tail; a launch after the tail where it is not fused) instead of on
  // the evaluation branch, so the training chain forks only once (after the fused forward)
  bool tail_metrics_ = false;
  // Phase 2 (enqueue_epoch): k_finalize -> k_wgrad -> k_adam and the train metrics as ONE launch
  // (k_lstm_tail, phase 2: the per-period sums relayed to the W_macro helpers, the moment
  // network's clip + Adam in the last blocks), DLAP_MOM_TAIL
  bool mom_tail_ = true;
  bool mom_adam_ = false;                    // set around enqueue_train_grads (enqueue_epoch)
  bool mom_tail_on(int phase) const {
    return phase == 2 && mom_tail_ && !xs_on_ && inv_code_.p != nullptr && splits_[0].set &&
           mom_tail_supported(md_, splits_[0].T);
  }
  bool mom_tail(int phase) const { return mom_adam_ && mom_tail_on(phase); }
  // phase 2: the LSTM recurrence once per run_epochs call (DLAP_P2_LSTM_CACHE)
  bool p2_lstm_cache_ = true;
  bool lstm_once_ = false;
  bool p2_lstm_cached() const {
    return p2_lstm_cache_ && md_.nrnn > 0 && (md_.nrnn == 1 || md_.dropout == 0.f) && !xs_on_;
  }
  bool tail_fused(int phase) const {
    return fused_tail_ && !xs_on_ && phase != 2 && splits_[0].set && lstm_tail_supported(md_, splits_[0].T);
  }
  // the pipelined eval-in-forward epoch: the clip + Adam update runs in the backward tail's last
  // blocks (k_lstm_tail, adam 2) after the evaluation branch's bookkeeping signalled, so the
  // training chain has no join edge and no k_adam launch (the branches join at the graph end)
  bool tail_adam_ = true;                    // DLAP_TAIL_ADAM
  bool tail_adam_pipe_ = false;              // DLAP_TAIL_ADAM=2: also in the one-graph fallback
  int tail_adam_mode_ = 0;                   // set around enqueue_train_grads (enqueue_pipe)
  float tail_lr_ = 0.f;
  // Co-residency guard: the tail's Adam blocks spin, holding their CU slots, until the
  // evaluation branch signals; G * nadam of them must leave at least half of the device's tail-sized
  // slots (occupancy query, tail_cap_) to the evaluation launches they wait for, else the epoch
  // keeps the join + k_adam update.
  bool adam_in_tail(int phase) const {
    if (!(tail_adam_ && tail_fused(phase) && inv_code_.p != nullptr)) return false;
    const int nadam = (md_.P_sdf + ADAM_PB - 1) / ADAM_PB;
    return tail_cap_ > 0 && 2 * G_ * nadam <= tail_cap_;
  }
  int tail_cap_ = 0;                         // k_lstm_tail workgroups resident at once (rebuild_jobs)
  // Split epoch graphs (the pipelined eval-in-forward epoch with the update in the tail): the
  // training chain is one single-queue graph on st_ (fused forward -> losses -> tower backward ->
  // tail + Adam) and the evaluation branch another on st2_ (k_wait_count -> evaluation towers ->
  // losses -> masks -> bookkeeping), launched side by side every epoch with NO graph edge between
  // them: the evaluation graph waits in-kernel for the fused forward's evaluation recurrences
  // (esync_ counts), the tail's Adam blocks for the bookkeeping's signal. A cross-queue edge
  // inside a graph costs ~5-6 us on the chain and a graph that ends on two queues ~12 us at its
  // boundary (profiles/r5_*timeline*); these cost one poll each.
  bool split_graphs_ = true;                 // DLAP_SPLIT_GRAPHS
  int unroll_ = 8;                           // DLAP_UNROLL: body epochs per split-graph launch
  double host_launch_s_ = 0.0;               // host time in the pipelined body launches ...
  long host_launch_n_ = 0;                   // ... over this many epochs (fused_info)
  int* fwd_esig_ = nullptr;                  // set around enqueue_train_grads (enqueue_chain_split)
  bool split_graphs(int phase) const {
    return split_graphs_ && adam_in_tail(phase) && (sep_eval(phase) || eval_rnn_in_fwd(phase));
  }
  // Split epoch graphs with the evaluation recurrences on the evaluation queue (DLAP_EVAL_SEP):
  // the training chain's fused forward runs the train recurrence only; the evaluation graph waits
  // for the previous update (k_wait_gen) and runs its own fused LSTM + tower forward (the
  // recurrences project their inputs, the towers trail the published periods). Bitwise equal to
  // the default; measured slower on the bench panel (0.153 vs 0.142 ms steady,
  // profiles/r6_eval_sep_ab.txt: the train-only fused forward still takes ~42 us, so it was not
  // bound by the evaluation recurrences, and the evaluation graph's own fused launch contends
  // with the chain) -- off by default.
  bool eval_sep_ = false;
  bool eval_sep_now_ = false;                // set around enqueue_eval_split (fused_eval)
  bool eval_selfproj_ = false;
  bool sep_eval(int phase) const {
    if (!eval_sep_ || phase == 2 || n_eval_jobs_ == 0 || !fused_fwd(phase) || md_.nrnn == 0 || md_.md.wide) return false;
    return mlp_fwd_rnn_supported(md_.md, md_.KS1, md_.WMB, md_.H, md_.nrnn, tmax_eval_) &&
           fused_grid(eval_grid(), n_eval_jobs_, cap_eval_) > 0;
  }
  void enqueue_chain_split(int phase, float lr) {
    tail_metrics_ = true;
    const bool sep = sep_eval(phase);
    tail_adam_mode_ = sep ? 3 : 2;
    tail_lr_ = lr;
    fwd_esig_ = sep ? nullptr : esync_.p;
    enqueue_train_grads(phase, true, 0, false, !sep);
    tail_metrics_ = false;
    tail_adam_mode_ = 0;
    fwd_esig_ = nullptr;
  }
  void enqueue_eval_split(int phase, int ignore_epoch, float sel) {      // captured on st2_
    if (sep_eval(phase)) {
      HTRACE("launch_wait_gen");
      launch_wait_gen(as<UpdJob>(j_upd_), G_, prog_limit_, st2_);
      eval_sep_now_ = true;
      // the recurrences project their own inputs when the towers skip the moment network (cached
      // moments); else k_proj first (gate projections + the moment bias table)
      eval_selfproj_ = self_proj_ && h_cache_;
      if (!eval_selfproj_) launch_proj(as<RnnJob>(j_rnn_eval_), n_eval_jobs_, tmax_eval_, dd(), md_, st2_, !h_cache_);
      enqueue_eval_towers(st2_);
      eval_sep_now_ = eval_selfproj_ = false;
    } else {
      HTRACE("launch_wait_count");
      launch_wait_count(esync_.p, ne_per_model() * G_, prog_limit_, prog_.p, G_, st2_);
      enqueue_eval_towers(st2_);
    }
    enqueue_dropmask(phase, 1, st2_);
    enqueue_epoch_end(phase, ignore_epoch, sel, st2_, 1);
  }
  void enqueue_train_tail(int phase) {
    const SplitDev& D = splits_[0];
    if (mom_tail(phase)) {
      HTRACE("launch_lstm_tail(phase 2)");
      launch_lstm_tail(as<UpdJob>(j_upd_), as<FinJob>(j_fin_), G_, dd(), md_, D.T, slab_stride(), st_,
                       loss_tab(2, false), 1, tail_lr_, 2);
      return;
    }
    const LossJob* lm = tail_metrics_ && phase != 2 ? loss_tab(phase, use_gram(phase)) : nullptr;
    if (tail_fused(phase)) {
      HTRACE("launch_lstm_tail");
      launch_lstm_tail(as<UpdJob>(j_upd_), as<FinJob>(j_fin_), G_, dd(), md_, D.T, slab_stride(), st_, lm,
                       tail_adam_mode_, tail_lr_);
      return;
    }
    if (lm) launch_job_metrics(lm, G_, st_);
    HTRACE("launch_finalize");
    launch_finalize(as<FinJob>(j_fin_), G_, dd(), md_, phase, slab_stride(), D.T, st_);
    // sharded: the rank-local tower gradients and per-period input gradients (dpp, or phase 2's
    // dab) summed over the ranks before the replicated LSTM backward / moment macro columns
    xs_call("grads", phase, st_);
    HTRACE("launch_lstm_bwd");
    launch_lstm_bwd(as<UpdJob>(j_upd_), G_, dd(), md_, D.T, phase, st_);
  }
  hipStream_t eval_prologue_hook_ = nullptr;   // see enqueue_train_grads
  void enqueue_train(int phase, float lr) {
    enqueue_train_grads(phase);
    HTRACE("launch_update");
    launch_update(as<UpdJob>(j_upd_), G_, dd(), md_, phase, lr, st_, inv_code_.p != nullptr);
  }
  void enqueue_eval(hipStream_t st) {
    enqueue_eval_prologue(st);
    enqueue_eval_towers(st);
  }
  void enqueue_eval_prologue(hipStream_t st) {
    if (n_eval_jobs_ == 0) return;
    HTRACE("launch_prologue");
    // fused: the input projections only, the recurrences run inside the tower launch
    if (fused_eval()) launch_proj(as<RnnJob>(j_rnn_eval_), n_eval_jobs_, tmax_eval_, dd(), md_, st, !h_cache_);
    else launch_prologue(as<RnnJob>(j_rnn_eval_), n_eval_jobs_, tmax_eval_, dd(), md_, st, !h_cache_);
  }
  void enqueue_eval_towers(hipStream_t st) {
    if (n_eval_jobs_ == 0) return;
    const int gx = eval_grid();
    if (md_.md.wide && zx_eval_) {     // layer 0 streamed inside the evaluation towers
      HTRACE("launch_mlp_fwd_zx");
      launch_mlp_fwd_zx(as<MlpJob>(j_mlp_eval_), n_eval_jobs_, std::max(1, zx_gx_ / n_eval_jobs_), md_.md, md_.WMB, st);
    } else {
      if (md_.md.wide)
        launch_proj0(as<WideJob>(j_wide_eval_), n_eval_jobs_, std::max(gx_proj_[1], gx_proj_[2]), md_.md, md_.WMB, st);
      HTRACE("launch_mlp_fwd");
      if (fused_eval())
        launch_mlp_fwd_rnn(as<MlpJob>(j_mlp_eval_), as<RnnJob>(j_rnn_eval_), dd(), n_eval_jobs_, fused_eval_gx(),
                           md_.md, md_.KS1, md_.WMB, md_.H, md_.nrnn, tmax_eval_, st, h_cache_, 0, eval_selfproj_);
      else
        launch_mlp_fwd(as<MlpJob>(j_mlp_eval_), n_eval_jobs_, gx, md_.md, md_.KS1, md_.WMB, st, h_cache_);
    }
    const bool eg = eval_gram_now();
    const LossJob* le = as<LossJob>(eg ? j_loss_eval_ : j_loss_eval_dense_);
    HTRACE("launch_period_fwd");
    period_fwd(le, n_eval_jobs_, tmax_eval_, st, false, 6);
    if (eg) {                        // quadratic-form terms per period (no asset passes)
      HTRACE("launch_period_bwd(eval)");
      launch_period_bwd(le, n_eval_jobs_, tmax_eval_, st);
    } else {
      HTRACE("launch_asset");
      launch_asset(le, n_eval_jobs_, nmax_eval_, md_.K, st);
      if (xs_on_) { launch_xs_loss_sums(le, n_eval_jobs_, st); xs_call("loss", 6, st); }
    }
    HTRACE("launch_job_metrics");
    launch_job_metrics(le, n_eval_jobs_, st);
  }
  void enqueue_epoch_end(int phase, int ignore_epoch, float sel, hipStream_t st, int signal = 0) {
    HTRACE("launch_epoch_end");
    launch_epoch_end(as<EpochJob>(j_epoch_[phase]), G_, phase, ignore_epoch, sel, md_.residual_factor,
                     md_.P, st, signal);
  }
  // sequential epoch: train step, evaluation, bookkeeping
  void enqueue_epoch(int phase, float lr, int ignore_epoch, float sel) {
    const bool mt = mom_tail_on(phase);
    mom_adam_ = mt;
    tail_lr_ = lr;
    enqueue_train_grads(phase);
    mom_adam_ = false;
    if (!mt) {
      HTRACE("launch_update");
      launch_update(as<UpdJob>(j_upd_), G_, dd(), md_, phase, lr, st_, inv_code_.p != nullptr);
    }
    if (phase != 2) { SoloScope solo(eval_solo_); enqueue_eval(st_); }
    enqueue_epoch_end(phase, ignore_epoch, sel, st_);
  }
  void enqueue_head(int phase, float lr) {
    enqueue_train_grads(phase);
    enqueue_dropmask(phase, 1, st_);                     // masks of the first pipelined epoch
    HTRACE("launch_update");
    launch_update(as<UpdJob>(j_upd_), G_, dd(), md_, phase, lr, st_, inv_code_.p != nullptr);
    // (k_adam does not count as a tail update: the first evaluation graph's wait passes)
    if (split_graphs(phase) && sep_eval(phase)) launch_gen_sync(as<UpdJob>(j_upd_), G_, st_);
  }
  // One-graph pipelined epoch (the split graphs' fallback: DLAP_SPLIT_GRAPHS=0, the update outside
  // the tail, or no fused forward): the training chain on st_, the evaluation branch forked
  // onto st2_ and joined before the update.
  void enqueue_pipe(int phase, float lr, int ignore_epoch, float sel) {
    HIP_OK(hipEventRecord(ev_fork_, st_));
    HIP_OK(hipStreamWaitEvent(st2_, ev_fork_, 0));
    if (eval_rnn_in_fwd(phase)) {
      // the evaluation recurrences run inside this epoch's fused training forward; the
      // evaluation branch forks after it: towers, losses, the bookkeeping and the next epoch's
      // dropout masks, beside the training backward and its tail (which computes the train
      // split's metrics)
      // (the one-graph fallback keeps the join + k_adam update unless DLAP_TAIL_ADAM=2: an
      // in-kernel wait across the graph's two branches would rest on the runtime mapping them
      // to different hardware queues -- ADVICE r5)
      const bool ta = tail_adam_pipe_ && adam_in_tail(phase);
      tail_metrics_ = true;
      tail_adam_mode_ = ta ? 2 : 0;
      tail_lr_ = lr;
      enqueue_train_grads(phase, true, 2, false, true);
      tail_metrics_ = false;
      tail_adam_mode_ = 0;
      HIP_OK(hipStreamWaitEvent(st2_, ev_a_, 0));
      enqueue_eval_towers(st2_);
      if (ta) {
        // the next epoch's masks, then the bookkeeping, whose signal releases the tail's update
        // (both read counters / parameters the update writes)
        enqueue_dropmask(phase, 1, st2_);
        enqueue_epoch_end(phase, ignore_epoch, sel, st2_, 1);
        HIP_OK(hipEventRecord(ev_join_, st2_));
        HIP_OK(hipStreamWaitEvent(st_, ev_join_, 0));
        return;
      }
      enqueue_epoch_end(phase, ignore_epoch, sel, st2_);
      enqueue_dropmask(phase, 1, st2_);
    } else {
      // training-chain nodes first (they land on the graph's first queue); the evaluation
      // branch's LSTM prologue right behind the training one (eval_prologue_hook_), so its
      // serial recurrence starts at the epoch start; this epoch's train metrics on the
      // evaluation branch after the loss pass (ev_mid_), then the bookkeeping and the masks
      eval_prologue_hook_ = st2_;
      enqueue_train_grads(phase, true, 0, true);
      eval_prologue_hook_ = nullptr;
      enqueue_eval_towers(st2_);
      if (phase != 2) {
        HIP_OK(hipStreamWaitEvent(st2_, ev_mid_, 0));
        launch_job_metrics(loss_tab(phase, use_gram(phase)), G_, st2_);
      }
      enqueue_epoch_end(phase, ignore_epoch, sel, st2_);
      enqueue_dropmask(phase, 1, st2_);
    }
    HIP_OK(hipEventRecord(ev_join_, st2_));
    HIP_OK(hipStreamWaitEvent(st_, ev_join_, 0));
    HTRACE("launch_update");
    launch_update(as<UpdJob>(j_upd_), G_, dd(), md_, phase, lr, st_, inv_code_.p != nullptr);
  }
  struct SoloScope {
    bool& f;
    explicit SoloScope(bool& x) : f(x) { f = true; }
    ~SoloScope() { f = false; }
  };
  void enqueue_tail(int phase, int ignore_epoch, float sel) {
    { SoloScope solo(eval_solo_); enqueue_eval(st_); }
    enqueue_epoch_end(phase, ignore_epoch, sel, st_);
  }
  template <typename F>
  hipGraphExec_t graph_for(const std::string& key, F&& enqueue, hipStream_t cs = nullptr) {
    if (!cs) cs = st_;
    auto it = graphs_.find(key);
    if (it != graphs_.end()) return it->second;
    const auto t_cap = std::chrono::steady_clock::now();
    hipGraph_t graph;
    {
      std::lock_guard<std::mutex> g(g_legacy_mu);
      HTRACE("capture %s tid=%ld", key.c_str(), (long)syscall(SYS_gettid));
      HIP_OK(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
      enqueue();
      HTRACE("end capture");
      HIP_OK(hipStreamEndCapture(cs, &graph));
    }
    HTRACE("instantiate");
    hipGraphExec_t exec;
    HIP_OK(hipGraphInstantiateWithFlags(&exec, graph, 0));
    HIP_OK(hipGraphDestroy(graph));
    // device-side upload now, not at the first launch (that launch may sit inside a timed or
    // latency-critical region)
    HIP_OK(hipGraphUpload(exec, cs));
    graphs_.emplace(key, exec);
    capture_s_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t_cap).count();
    return exec;
  }
  void fwd_only(int s, bool train_mode, bool do_mom, bool wait) {
    const SplitDev& D = splits_[s];
    if (!D.set) throw std::runtime_error("split not set");
    join_eval_gram();
    // job tables of (split, mode) for every model, built once per rebuild (module API calls
    // issue no host allocation / synchronous copy). The train split keeps its LSTM state
    // (final (h, c) of every layer for the module API).
    const int key = s * 4 + (train_mode ? 2 : 0) + (do_mom ? 1 : 0);
    FwdTables& F = fwd_tables_[key];
    if (!F.built) {
      std::vector<RnnJob> rj;
      std::vector<MlpJob> mj;
      std::vector<LossJob> lj;
      std::vector<WideJob> wj;
      for (int g = 0; g < G_; ++g) {
        rj.push_back(rnn_job(g, s, train_mode, s == 0 ? 1 : 0));
        mj.push_back(mlp_job(g, s, train_mode, true, do_mom));
        lj.push_back(loss_job(g, s, 0));
        wj.push_back(wide_job(g, s, true, do_mom));
        if (!do_mom) lj.back().h = nullptr;
      }
      upload(F.r, rj); upload(F.m, mj); upload(F.l, lj); upload(F.w, wj);
      F.built = true;
    }
    DevBuf<char>& a = F.r;
    DevBuf<char>& b = F.m;
    DevBuf<char>& c = F.l;
    DevBuf<char>& w = F.w;
    const bool zx = md_.md.wide && zx_eval_ && !train_mode;
    if (md_.md.wide && !zx) launch_proj0(as<WideJob>(w), G_, gx_proj_[s], md_.md, md_.WMB, st_);
    launch_prologue(as<RnnJob>(a), G_, D.T, dd(), md_, st_, do_mom);
    if (zx) launch_mlp_fwd_zx(as<MlpJob>(b), G_, std::max(1, zx_gx_ / G_), md_.md, md_.WMB, st_);
    else launch_mlp_fwd(as<MlpJob>(b), G_, gx_fwd_[s], md_.md, md_.KS1, md_.WMB, st_);
    period_fwd(as<LossJob>(c), G_, D.T, st_, true, 1 << s);
    launch_asset(as<LossJob>(c), G_, D.N, md_.K, st_);
    if (xs_on_) { launch_xs_loss_sums(as<LossJob>(c), G_, st_); xs_call("loss", 1 << s, st_); }
    launch_job_metrics(as<LossJob>(c), G_, st_);
    if (wait) sync();
  }
};

// Native-frame backtrace on a host crash (failure detection): Python's faulthandler
// only names the Python frame; this prints the native frames (file-relative offsets, resolvable
// with addr2line against the in-tree .so) and then chains to the previous handler.
static struct sigaction g_prev_segv, g_prev_bus;
static void dlap_crash_handler(int sig, siginfo_t*, void*) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  static const char msg[] = "[dlap] native backtrace:\n";
  (void)!write(2, msg, sizeof msg - 1);
  backtrace_symbols_fd(fr, n, 2);
  sigaction(sig, sig == SIGBUS ? &g_prev_bus : &g_prev_segv, nullptr);
  raise(sig);
}
static void install_crash_handler() {
  if (env_int("DLAP_CRASH_TRACE", 1) == 0) return;
  struct sigaction cur {};
  if (sigaction(SIGSEGV, nullptr, &cur) == 0 && (cur.sa_flags & SA_SIGINFO) &&
      cur.sa_sigaction == dlap_crash_handler)
    return;                                    // (re-installed on entry points: others may replace it)
  struct sigaction sa {};
  sa.sa_sigaction = dlap_crash_handler;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, &g_prev_segv);
  sigaction(SIGBUS, &sa, &g_prev_bus);
}

// DLAP_EMBED: the host-ASan harness (csrc/host/asan_main.cpp) links the engine into an
// executable that embeds Python; the module is then a built-in one.
#ifdef DLAP_EMBED
#include <pybind11/embed.h>
PYBIND11_EMBEDDED_MODULE(_dlap_hip, m) {
#else
PYBIND11_MODULE(_dlap_hip, m) {
#endif
  install_crash_handler();
  m.doc() = "DLAP MI355X native engine (HIP kernels for gfx950 + hipGraph epoch executor)";
  py::class_<Engine>(m, "Engine")
      .def(py::init<int, int, int, int, bool, std::vector<int>, std::vector<int>, int, float, bool, bool,
                    float, int, int, bool>(),
           py::arg("F"), py::arg("M"), py::arg("nrnn"), py::arg("H"), py::arg("raw_macro_sdf"),
           py::arg("hidden"), py::arg("mom_hidden"), py::arg("K"), py::arg("dropout"),
           py::arg("normalize_w"), py::arg("weighted"), py::arg("residual"), py::arg("G"),
           py::arg("max_epochs"), py::arg("fp32") = false)
      .def("describe", &Engine::describe)
      .def("set_split", &Engine::set_split)
      .def("set_split_dev", &Engine::set_split_dev)
      .def("set_split_dense", &Engine::set_split_dense, py::arg("s"), py::arg("feats"), py::arg("ret"),
           py::arg("mask"), py::arg("mask_bool"), py::arg("macro"), py::arg("T"), py::arg("N"), py::arg("F"),
           py::arg("stream") = 0)
      .def("read_split", &Engine::read_split)
      .def("set_params", &Engine::set_params)
      .def("get_params", &Engine::get_params)
      .def("get_grads", &Engine::get_grads)
      .def("get_snapshot", &Engine::get_snapshot)
      .def("load_snapshot", &Engine::load_snapshot)
      .def("set_seed", &Engine::set_seed)
      .def("set_tower_salt", &Engine::set_tower_salt)
      .def("get_opt_state", &Engine::get_opt_state)
      .def("set_opt_state", &Engine::set_opt_state)
      .def("get_tracker_state", &Engine::get_tracker_state)
      .def("set_tracker_state", &Engine::set_tracker_state)
      .def("begin_phase", &Engine::begin_phase)
      .def("snap_flags", &Engine::snap_flags)
      .def("epoch_count", &Engine::epoch_count)
      .def("history", &Engine::history)
      .def("run_epochs", &Engine::run_epochs, py::call_guard<py::gil_scoped_release>())
      .def("set_pipeline", &Engine::set_pipeline)
      .def("set_safe_mode", &Engine::set_safe_mode)
      .def("plan_phase", &Engine::plan_phase)
      .def("gram_plan", &Engine::gram_plan)
      .def("set_lr", &Engine::set_lr)
      .def("set_dropout", &Engine::set_dropout)
      .def("get_dropout", &Engine::get_dropout)
      .def_static("blocking_calls", []() { return (long long)g_blocking.load(); })
      .def_static("live_engines", []() { return g_live_engines.load(); })
      .def_static("rnn_timestamps", []() { return rnn_timestamps(); })
      .def("fused_forward", [](Engine& e, int phase) { e.ensure_jobs(); return e.fused_fwd(phase); })
      .def("prog_timeouts", &Engine::prog_timeouts)
      .def("reset_prog_errors", &Engine::reset_prog_errors)
      .def("fused_info", [](Engine& e) { e.ensure_jobs(); return e.fused_info(); })
      .def("capture_seconds", [](Engine& e) { return e.capture_seconds(); })
      .def_static("loss_timestamps", []() { return loss_timestamps(); })
      .def_static("mlp_timestamps", []() { return mlp_timestamps(); })
      .def_static("tbwd_timestamps", []() { return tbwd_timestamps(); })
      .def("set_xs", &Engine::set_xs)
      .def("xs_set_globals", &Engine::xs_set_globals)
      .def("ws_ptr", &Engine::ws_ptr)
      .def("grads_ptr", &Engine::grads_ptr)
      .def("forward_split", &Engine::forward_split, py::arg("s"), py::arg("train_mode"), py::arg("do_mom"),
           py::arg("wait") = true)
      .def("train_step", &Engine::train_step)
      .def("backward_only", &Engine::backward_only, py::arg("phase"), py::arg("wait") = true)
      .def("set_stream", &Engine::set_stream, py::arg("stream"), py::arg("external") = true)
      .def("set_params_dev", &Engine::set_params_dev)
      .def("join_from", &Engine::join_from)
      .def("xs_backward", &Engine::xs_backward, py::arg("phase"), py::arg("dw"), py::arg("dE"), py::arg("sdf"),
           py::arg("dh") = 0)
      .def("set_hidden", &Engine::set_hidden)
      .def("copy_hidden_grad", &Engine::copy_hidden_grad)
      .def("split_rows", &Engine::split_rows)
      .def("join_to", &Engine::join_to)
      .def("set_drop_step", &Engine::set_drop_step)
      .def("copy_ws", &Engine::copy_ws)
      .def("copy_grads", &Engine::copy_grads)
      .def("copy_hidden", &Engine::copy_hidden)
      .def("read_ws", &Engine::read_ws)
      .def("read_aux", &Engine::read_aux)
      .def("read_gram", &Engine::read_gram)
      .def("refresh_gram", &Engine::refresh_gram)
      .def("gram_enabled", &Engine::gram_enabled)
      .def("read_blob", &Engine::read_blob)
      .def("sync", &Engine::sync, py::call_guard<py::gil_scoped_release>())
      .def("stream", &Engine::stream);
  m.def("ensemble_portfolios",
        [](uintptr_t W, int G, int T, int N, uintptr_t R, uintptr_t mask, uintptr_t port, uintptr_t port_ind,
           uintptr_t stream) {
          launch_ensemble(reinterpret_cast<const float*>(W), G, T, N, reinterpret_cast<const float*>(R),
                          reinterpret_cast<const float*>(mask), reinterpret_cast<float*>(port),
                          reinterpret_cast<float*>(port_ind), reinterpret_cast<hipStream_t>(stream));
        },
        "K11: ensemble portfolio [T] and individual portfolios [G][T] from gathered weights (device pointers)");
  m.attr("HIST_W") = (int)HIST_W;
  m.attr("SC_NSCAL") = (int)SC_NSCAL;
}
