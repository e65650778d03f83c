// Macro-state LSTM forward / backward and the moment network's per-period macro bias.
//
// Replaces `MacroLSTM.forward` = one nn.LSTM over the whole T-sequence with batch 1
// (`/root/reference/src/model.py:21-84`) and the macro half of the moment
// input concatenation (`model.py:513-516`).
//   * PyTorch gate order i, f, g, o and both biases (state_dict compatible);
//   * zero initial state for every split (the reference passes hidden=None everywhere);
//   * inter-layer dropout on every layer output but the last (torch semantics), train only.
//
// Kernels
//   k_proj      grid (ceil(T/16), jobs): the layer-0 input projection of every step
//               xg[t] = W_ih x_t + b_ih + b_hh and the moment table
//               abias[t][c] = W_m0[c, :M] . m_t + b_m0[c]  (zero-padded to 64 columns);
//               the weights are staged in LDS, each thread owns one output for 4 periods.
//   k_lstm      one wave per job: the recurrence. Lane k owns hidden unit k and keeps its
//               4 rows of W_hh (and W_ih for layers > 0) in registers; h_{t-1} is broadcast
//               with v_readlane (no LDS, no barrier); xg is staged in LDS when it fits.
//   k_lstm_bwd  one workgroup per model: BPTT on wave 0 (same ownership, dgates broadcast
//               with v_readlane), then every thread reduces the weight gradients over t
//               from LDS-staged dgates (thread per macro column: 4H FMAs per load).
//               Phase 2 instead builds the moment layer-0 macro-column / bias gradients.
#include <algorithm>
#include <cstdlib>
#include "common.h"
#include "layout.h"
#include "rnn.h"
#include "update.h"
#include "lstm_gls.h"
#include "finalize.h"
#include "loss_dev.h"
#include "pack_dev.h"

#define DLAP_MAX_M 1024

// In-kernel phase timestamps (wall clock, 100 MHz) for profiling the serial kernels, read by
// Engine.rnn_timestamps(). Slots: [0..3] k_lstm_gl train launch, [4..7] its eval launch (last
// block = longest split), [8..12] k_lstm_bwd.
__device__ long long g_rnn_ts[24];   // [16]: fused tail, dpp in LDS; [17]: W_ih start
#define RNN_TS(slot, cond) do { if ((cond) && threadIdx.x == 0) g_rnn_ts[slot] = wall_clock64(); } while (0)

// Fast activations (v_exp + v_rcp): |err| < 1e-6 relative in the ranges that matter; tanh
// switches to its cubic Taylor form near 0 where 2*sigm(2x)-1 would cancel.
DLAP_DEV float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
DLAP_DEV float ftanh(float x) {
  const float t = 2.f * sigm(2.f * x) - 1.f;
  return fabsf(x) < 0.0125f ? x * (1.f - x * x * (1.f / 3.f)) : t;
}

// ------------------------------------------------------------------------ k_proj -------
// (proj_tile: lstm_gls.h)
// grid (ceil(T/16), column tiles, jobs); blockIdx.y counts from column tile y0 (y0 = G4/16 when
// the LSTM projects its own inputs: only the moment table is left here).
__global__ __launch_bounds__(64) void k_proj(const RnnJob* __restrict__ jobs,
                                             const ModelDesc* __restrict__ md, int y0) {
  const RnnJob& J = jobs[blockIdx.z];
  const int T = J.T;
  const int t0 = blockIdx.x * 16, o0 = (blockIdx.y + y0) * 16;
  const int G4 = md->nrnn > 0 ? 4 * md->H : 0;
  if (t0 >= T) return;
  if (o0 >= G4 && !J.abias) return;
  const bool tsm = blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0;
  RNN_TS(12, tsm);
  // the fused forward's progress counter starts from zero (read only by kernels after this one)
  if (J.prog && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) gp(J.prog)[0] = 0;
  const f32x4 acc = proj_tile(J, md, t0, o0);
  const int l = threadIdx.x, n = l & 15, kq = l >> 4;
  const int o = o0 + n;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int t = t0 + 4 * kq + r;
    if (t >= T) break;
    const float v = acc[r];
    if (o < G4) gp(J.xg)[(size_t)t * G4 + o] = v;
    else if (o - G4 < 64) gp(J.abias)[t * 64 + (o - G4)] = v;
  }
  RNN_TS(14, tsm);
}


// BPTT coefficients of one (t, unit), computed by k_lstm_bwd in a parallel pre-pass from the
// saved gates / cells, so that the serial backward recurrence is only
//   dh = dout + dh_next; dc = dh*A + dc_next; d_q = dc*B_q (d_o = dh*B_o); dc_next = dc*F;
//   dh_next = W_hh^T d.
// Layout [t][6][H]: A = o (1 - tanh(c)^2), Bi = g i (1 - i), Bf = c_prev f (1 - f),
// Bg = i (1 - g^2), Bo = tanh(c) o (1 - o), F = f.
#define LSTM_NCOEF 6
#define LSTM_GSEG 8        // max time segments of the k_lstm_bwd weight-gradient sums

// ------------------------------------------------------------------------ k_lstm -------
// STAGE: layer-0 input projections staged in LDS (T*4H <= 12288). The layer-0 and deeper
// layer loops are separate and fully unrolled over HM (>= H; padded units have zero weights,
// so they stay at h = c = 0 and contribute nothing): the time loop has no branches, no
// memory loads outside LDS, and only fire-and-forget global stores, so nothing on the serial
// chain waits on HBM.
template <int HM, bool STAGE>
__global__ __launch_bounds__(64) void k_lstm(const RnnJob* __restrict__ jobs,
                                             const ModelDesc* __restrict__ md) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const RnnJob& J = jobs[blockIdx.x];
  const int nrnn = md->nrnn;
  if (nrnn == 0) return;
  const int T = J.T, H = md->H, G4 = 4 * H;
  const int lane = threadIdx.x;
  const bool act = lane < H;
  const int k = act ? lane : 0;
  const bool drop = J.train && J.dropout > 0.f;
  const uint32_t thr = (uint32_t)(J.dropout * 16777216.f + 0.5f);
  const float scale = drop ? 1.f / (1.f - J.dropout) : 1.f;
  const uint32_t step = J.step ? (uint32_t)*gp(J.step) : 0u;
  const auto params = gp(J.params);
  const auto xg = gp(J.xg);
  const bool save = J.sc != nullptr;
  for (int l = 0; l < nrnn; ++l) {
    const auto Whh = params + md->lstm_w_hh[l];
    float whh[4][HM], wih[4][HM], bias[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int j = 0; j < HM; ++j) {
        const bool ok = act && j < H;
        const int jj = j < H ? j : 0;
        const float a = Whh[(q * H + k) * H + jj];
        const float b = l > 0 ? params[md->lstm_w_ih[l] + (q * H + k) * H + jj] : 0.f;
        whh[q][j] = ok ? a : 0.f;
        wih[q][j] = ok ? b : 0.f;
      }
      const float bb = l > 0 ? params[md->lstm_b_ih[l] + q * H + k] + params[md->lstm_b_hh[l] + q * H + k] : 0.f;
      bias[q] = act ? bb : 0.f;
    }
    if (STAGE && l == 0) {
      for (int i = lane; i < T * G4; i += 64) sm[i] = xg[i];
      __syncthreads();
    }
    const auto hout = save ? gp(J.sh) + (size_t)l * T * H : gp(J.out);
    const auto sg = gp(J.sg) + (size_t)l * T * G4;
    const auto sc = gp(J.sc) + (size_t)l * T * H;
    float h = act && J.h0 ? gp(J.h0)[l * H + k] : 0.f, c = act && J.c0 ? gp(J.c0)[l * H + k] : 0.f;
    auto cell = [&](int t, const float (&p)[4]) {
      const float gi = sigm(p[0]), gf = sigm(p[1]), gg = ftanh(p[2]), go = sigm(p[3]);
      c = gf * c + gi * gg;
      h = go * ftanh(c);
      if (act) {
        hout[(size_t)t * H + k] = h;
        if (save) {
          sc[(size_t)t * H + k] = c;
          const auto g = sg + (size_t)t * G4;
          g[k] = gi; g[H + k] = gf; g[2 * H + k] = gg; g[3 * H + k] = go;
        }
      }
    };
    if (l == 0) {
      auto ldx = [&](int t, float (&v)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float x = STAGE ? sm[t * G4 + q * H + k] : xg[(size_t)t * G4 + q * H + k];
          v[q] = act ? x : 0.f;
        }
      };
      float nx[4];
      ldx(0, nx);
      for (int t = 0; t < T; ++t) {
        float p[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) p[q] = nx[q];
        ldx(t + 1 < T ? t + 1 : t, nx);                // prefetch the next step's inputs
#pragma unroll
        for (int q = 0; q < 4; ++q) p[q] += bcast_dot<HM>(whh[q], h);
        cell(t, p);
      }
    } else {
      const auto xin = gp(J.xin);                   // layer l-1 output (dropout on read)
      const uint32_t key_in = dropout_key(J.seed, step, 32 + (l - 1));
      float nxv = act ? xin[k] : 0.f;
      for (int t = 0; t < T; ++t) {
        float xv = nxv;
        nxv = act ? xin[(size_t)(t + 1 < T ? t + 1 : t) * H + k] : 0.f;
        if (drop) xv = dropout_keep(key_in, (uint32_t)t, (uint32_t)k, thr) ? xv * scale : 0.f;
        float p[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) p[q] = bias[q] + bcast_dot<HM>(wih[q], xv) + bcast_dot<HM>(whh[q], h);
        cell(t, p);
      }
    }
    __threadfence_block();
    if (l + 1 < nrnn) {
      const auto xin = gp(J.xin);
      for (int i = lane; i < T * H; i += 64) xin[i] = hout[i];
      __threadfence_block();
    } else if (save) {
      const auto out = gp(J.out);
      for (int i = lane; i < T * H; i += 64) out[i] = hout[i];
    }
  }
}

// ----------------------------------------------------------------------- k_lstm_gl -----
// Gate-per-lane recurrence for 4H <= 64: lane L owns gate row L (q = L / H, unit L % H), so a
// step is HM broadcast FMAs + ONE activation per lane (sigmoid, or tanh = 2 sigm(2x) - 1 on
// the g rows) instead of four per unit lane; the f/g/o values are then gathered onto the unit
// lanes (DPP row rotates when 4H <= 16, ds_bpermute otherwise). ~3x fewer instructions on
// the serial chain than the unit-per-lane form. EXACT = HM is H itself (DPP offsets need it).
template <int CTRL>
DLAP_DEV float dppf(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}

template <int HM, bool DPPG, bool STAGE>
__global__ __launch_bounds__(64) void k_lstm_gl(const RnnJob* __restrict__ jobs,
                                                const ModelDesc* __restrict__ md) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const RnnJob& J = jobs[blockIdx.x];
  const int nrnn = md->nrnn;
  if (nrnn == 0) return;
  const int T = J.T, H = DPPG ? HM : md->H, G4 = 4 * H;
  const int L = threadIdx.x;
  const bool gl = L < G4;                 // lane owns gate row L
  const bool ul = L < H;                  // lane owns unit L (cell state, output)
  const int row = gl ? L : 0;
  const bool is_g = gl && L >= 2 * H && L < 3 * H;
  const float ka = is_g ? 2.f : 1.f;      // act(x) = kb * sigm(ka x) + kc
  const float kb = is_g ? 2.f : 1.f, kc = is_g ? -1.f : 0.f;
  const bool drop = J.train && J.dropout > 0.f;
  const uint32_t thr = (uint32_t)(J.dropout * 16777216.f + 0.5f);
  const float scale = drop ? 1.f / (1.f - J.dropout) : 1.f;
  const uint32_t step = J.step ? (uint32_t)*gp(J.step) : 0u;
  const auto params = gp(J.params);
  const auto xg = gp(J.xg);
  const bool save = J.sc != nullptr;
  const int tsb = save ? 0 : 4;
  const bool tsm = save || blockIdx.x == gridDim.x - 1;
  RNN_TS(tsb + 0, tsm);
  for (int l = 0; l < nrnn; ++l) {
    float whh[HM], wih[HM];
#pragma unroll
    for (int j = 0; j < HM; ++j) {
      const bool ok = gl && j < H;
      const int jj = j < H ? j : 0;
      const float a = params[md->lstm_w_hh[l] + row * H + jj];
      const float b = l > 0 ? params[md->lstm_w_ih[l] + row * H + jj] : 0.f;
      whh[j] = ok ? a : 0.f;
      wih[j] = ok ? b : 0.f;
    }
    const float bb = l > 0 ? params[md->lstm_b_ih[l] + row] + params[md->lstm_b_hh[l] + row] : 0.f;
    const float bias = gl ? bb : 0.f;
    if (STAGE && l == 0) {
      for (int i = L; i < T * G4; i += 64) sm[i] = xg[i];
      __syncthreads();
    }
    if (l == 0) RNN_TS(tsb + 1, tsm);
    const auto hout = save ? gp(J.sh) + (size_t)l * T * H : gp(J.out);
    const auto sg = gp(J.sg) + (size_t)l * T * G4;
    const auto sc = gp(J.sc) + (size_t)l * T * H;
    const auto out = gp(J.out);
    const bool last = l + 1 == nrnn;
    float h = ul && J.h0 ? gp(J.h0)[l * H + L] : 0.f, c = ul && J.c0 ? gp(J.c0)[l * H + L] : 0.f;
    auto cell = [&](int t, float pre) {
      pre += bcast_dot<HM>(whh, h);
      float y = kb * sigm(ka * pre) + kc;
      if (is_g && fabsf(pre) < 0.0125f) y = pre * (1.f - pre * pre * (1.f / 3.f));
      const float gf = gl_gather<HM, DPPG>(y, H, 1);
      const float gg = gl_gather<HM, DPPG>(y, 2 * H, 2);
      const float go = gl_gather<HM, DPPG>(y, 3 * H, 3);
      c = gf * c + y * gg;                 // y = i on the unit lanes
      h = ul ? go * ftanh(c) : 0.f;
      if (save && gl) sg[(size_t)t * G4 + L] = y;
      if (ul) {
        hout[(size_t)t * H + L] = h;
        if (save) {
          sc[(size_t)t * H + L] = c;
          if (last) out[(size_t)t * H + L] = h;      // the tower input, no copy pass
        }
      }
    };
    if (l == 0) {
      float nx = gl ? (STAGE ? sm[L] : xg[L]) : 0.f;
      for (int t = 0; t < T; ++t) {
        const float pre = nx;
        const int tn = t + 1 < T ? t + 1 : t;            // prefetch the next step's input
        const float v = STAGE ? sm[tn * G4 + row] : xg[(size_t)tn * G4 + row];
        nx = gl ? v : 0.f;
        cell(t, pre);
      }
    } else {
      const auto xin = gp(J.xin);                        // layer l-1 output (dropout on read)
      const uint32_t key_in = dropout_key(J.seed, step, 32 + (l - 1));
      float nxv = ul ? xin[L] : 0.f;
      for (int t = 0; t < T; ++t) {
        float xv = nxv;
        const float v = xin[(size_t)(t + 1 < T ? t + 1 : t) * H + (ul ? L : 0)];
        nxv = ul ? v : 0.f;
        if (drop) xv = dropout_keep(key_in, (uint32_t)t, (uint32_t)(ul ? L : 0), thr) ? xv * scale : 0.f;
        float pre = bias;
#pragma unroll
        for (int j = 0; j < HM; ++j)
          pre += wih[j] * __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xv), j));
        cell(t, pre);
      }
    }
    if (l == 0) RNN_TS(tsb + 2, tsm);
    __threadfence_block();
    if (l + 1 < nrnn) {
      const auto xin = gp(J.xin);
      for (int i = L; i < T * H; i += 64) xin[i] = hout[i];
      __threadfence_block();
    }
  }
  RNN_TS(tsb + 3, tsm);
}

// ---------------------------------------------------------------------- k_lstm_gls -----
// k_lstm_gl with every per-step output kept in LDS (lstm_gls.h): one wave per job.
template <int HM, bool DPPG>
__global__ __launch_bounds__(64) void k_lstm_gls(const RnnJob* __restrict__ jobs, const ModelDesc* __restrict__ md) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const RnnJob& J = jobs[blockIdx.x];
  if (md->nrnn == 0) return;
  const int tsb = J.sc != nullptr ? 0 : 4;
  const bool tsm = J.sc != nullptr || blockIdx.x == gridDim.x - 1;
  RNN_TS(tsb + 0, tsm);
  lstm_gls_body<HM, DPPG, true, false>(J, md, sm, nullptr, tsm ? g_rnn_ts : nullptr, tsb);
}

static const bool g_rtrace = [] { const char* v = std::getenv("DLAP_TRACE_HOST"); return v && *v == '1'; }();
#define RTRACE(...) do { if (g_rtrace) { fprintf(stderr, "[dlap-trace] " __VA_ARGS__); fputc('\n', stderr); fflush(stderr); } } while (0)

void launch_proj(const RnnJob* jobs, int njobs, int tmax, const ModelDesc* md, const ModelDesc& mh,
                 hipStream_t st, bool abias) {
  const int G4 = mh.nrnn > 0 ? 4 * mh.H : 0;
  const int ny = abias ? mh.proj_np / 16 : (G4 + 15) / 16;
  RTRACE("proj jobs=%p njobs=%d tmax=%d ny=%d st=%p", (const void*)jobs, njobs, tmax, ny, (void*)st);
  if (ny <= 0) return;
  hipLaunchKernelGGL(k_proj, dim3((tmax + 15) / 16, ny, njobs), dim3(64), 0, st, jobs, md, 0);
  HIP_OK(hipGetLastError());
}

void launch_prologue(const RnnJob* jobs, int njobs, int tmax, const ModelDesc* md, const ModelDesc& mh,
                     hipStream_t st, bool abias, bool lstm) {
  // k_proj: the layer-0 gate projections (unless only the moment bias is asked for) and, with
  // abias, the moment network's per-period bias table; then the recurrence: the gate-per-lane
  // form with its outputs in LDS (k_lstm_gls) when they fit in 64 KiB, the same form with
  // global outputs (k_lstm_gl: long splits) otherwise, and the unit-per-lane form (k_lstm) for
  // H > 16
  const int G4 = mh.nrnn > 0 ? 4 * mh.H : 0;
  const int y0 = abias && !lstm ? G4 / 16 : 0;
  const int ny = abias ? mh.proj_np / 16 - y0 : (lstm ? (G4 + 15) / 16 : 0);
  RTRACE("prologue jobs=%p njobs=%d tmax=%d H=%d nrnn=%d proj_np=%d y0=%d ny=%d st=%p", (const void*)jobs,
         njobs, tmax, mh.H, mh.nrnn, mh.proj_np, y0, ny, (void*)st);
  if (ny > 0) {
    hipLaunchKernelGGL(k_proj, dim3((tmax + 15) / 16, ny, njobs), dim3(64), 0, st, jobs, md, y0);
    HIP_OK(hipGetLastError());
  }
  RTRACE("prologue proj launched");
  if (mh.nrnn > 0 && lstm) {
    const bool stage = tmax * 4 * mh.H <= 12288;     // 48 KiB of LDS
    const size_t sh = stage ? (size_t)tmax * 4 * mh.H * sizeof(float) : 0;
    const bool gls = mh.H <= 16 && gls_lds_floats(tmax, mh.H) * sizeof(float) <= 64 * 1024;
    const size_t shg = gls_lds_floats(tmax, mh.H) * sizeof(float);
#define G_CASE(HM, DP) \
    if (stage) hipLaunchKernelGGL((k_lstm_gl<HM, DP, true>), dim3(njobs), dim3(64), sh, st, jobs, md); \
    else hipLaunchKernelGGL((k_lstm_gl<HM, DP, false>), dim3(njobs), dim3(64), sh, st, jobs, md);
#define S_CASE(HM, DP) hipLaunchKernelGGL((k_lstm_gls<HM, DP>), dim3(njobs), dim3(64), shg, st, jobs, md);
    if (gls) {
      if (mh.H == 1) { S_CASE(1, true) } else if (mh.H == 2) { S_CASE(2, true) }
      else if (mh.H == 3) { S_CASE(3, true) } else if (mh.H == 4) { S_CASE(4, true) }
      else if (mh.H <= 8) { S_CASE(8, false) } else { S_CASE(16, false) }
    } else if (mh.H == 1) { G_CASE(1, true) } else if (mh.H == 2) { G_CASE(2, true) }
    else if (mh.H == 3) { G_CASE(3, true) } else if (mh.H == 4) { G_CASE(4, true) }
    else if (mh.H <= 8) { G_CASE(8, false) } else if (mh.H <= 16) { G_CASE(16, false) }
    else if (stage) hipLaunchKernelGGL((k_lstm<32, true>), dim3(njobs), dim3(64), sh, st, jobs, md);
    else hipLaunchKernelGGL((k_lstm<32, false>), dim3(njobs), dim3(64), sh, st, jobs, md);
#undef G_CASE
#undef S_CASE
    HIP_OK(hipGetLastError());
    RTRACE("prologue lstm launched (gls=%d shg=%zu)", (int)gls, shg);
  }
}

// -------------------------------------------------------------------- k_lstm_bwd -------
// grid: models, 256 threads. BPTT through every LSTM layer (phases 1/3). Per layer the saved
// gates / cells / outputs and the incoming gradient are staged in LDS, the recurrence runs
// on wave 0 from LDS (next step prefetched), then all threads form the small gradients
// (W_hh, biases, W_ih of layers > 0, d input of the layer below). The layer-0 W_ih
// gradient (T x 4H x M) is left to k_wgrad, which has many workgroups.
// Dense-state BPTT (H = 4, `scan`): the backward recurrence is LINEAR in the carried state
// y_t = (dh_t, dc_next_t) in R^8 (dh_t = dout_t + dh_next, the cell gradient arriving from t+1):
//   y_t = M_{t+1} y_{t+1} + (dout_t, 0),   M_t = [[Pc diag(A) + Qo, Pc], [diag(F A), diag(F)]],
//   Pc[j][k] = sum_{q = i,f,g} W_hh[4q+k][j] B_q[k],  Qo[j][k] = W_hh[12+k][j] Bo[k]
// (A, B_q, F: the pre-pass coefficients of step t). All M_t are formed in parallel, and the
// serial chain is one 8x8 mat-vec per step on one wave, lane (i, j) = 8 i + j holding M[i][j]:
// the product is reduced over j inside 8-lane groups (DPP quad perms + half mirror, "R layout":
// every lane of group i holds y[i]) on even steps and over i across the wave (DPP row_ror 8 +
// v_permlane16_swap + v_permlane32_swap, "C layout": lane (i, j) holds y[j]) on odd steps --
// each layout is the other's input layout, so no lane permutation is on the chain. ~6 VALU per
// step instead of the gate-per-lane step's ~25 (one dependent 4-unit cell update + a 16-lane
// reduce-scatter). The gate gradients then follow from the recorded y_t in parallel.
// m * y rounded once and hidden from the combiner: p + dpp(p) must not become fma(m, y, dpp(p))
// (the lanes of a group would then round differently and disagree on y)
DLAP_DEV float rmul(float m, float y) {
  float p = m * y;
  asm volatile("" : "+v"(p));
  return p;
}
DLAP_DEV float red8_j(float p) {         // sum over the 8 lanes of a group (lanes 8i .. 8i+7)
  p += dppf<0xB1>(p);                    // quad_perm [1,0,3,2]
  p += dppf<0x4E>(p);                    // quad_perm [2,3,0,1]
  p += dppf<0x141>(p);                   // row_half_mirror: lane j <-> 7 - j (the other quad)
  return p;
}
DLAP_DEV float red8_i(float p) {         // sum over lanes j, j+8, ..., j+56
  p += dppf<0x128>(p);                   // row_ror:8 = lane ^ 8 inside a 16-lane row
  {
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(p), __float_as_uint(p), false, false);
    p = __uint_as_float(s[0]) + __uint_as_float(s[1]);      // lane ^ 16
  }
  {
    const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(p), __float_as_uint(p), false, false);
    p = __uint_as_float(s[0]) + __uint_as_float(s[1]);      // lane ^ 32
  }
  return p;
}
// weight-gradient partials: segment sums [S][nout], or the four MFMA tiles of the H = 4 path
__host__ __device__ inline size_t lstm_gpart_floats(int H) {
  const size_t a = 256 + (size_t)16 * H * (2 * H + 1);
  return a > 1024 ? a : 1024;
}
// LDS floats of the dense-state path: M_t [T][64], y_t [T][8], W_hh [64], pair maps N_t / v_t
__host__ __device__ inline size_t lstm_bwd_scan_floats(int T) { return (size_t)T * 72 + 64 + (size_t)((T - 1) / 2) * 72; }

// LDS map of the LSTM backward (float offsets). k_lstm_bwd: coefficients, layer outputs,
// incoming gradient, gate gradients, junk slots, weight-gradient partials, then (dense-state
// path) M_t, y_t, W_hh, the pair maps. The fused tail (k_lstm_tail, `fused`): the step matrices
// M_t live in global scratch (UpdJob::mscr) and the pair maps share one region with the gate
// gradients + partials (dead before those are formed), so the block fits two per CU beside
// the finalisation blocks of the same launch.
struct LstmBwdLds { size_t cf, h, d, dgs, junk, gpart, M, y, W, N, v, total; };
// hand-off words of the fused tail (UpdJob::tail_ctr, one 128-byte line each): periods published,
// gate gradients published, W_ih helper blocks done
__host__ __device__ inline LstmBwdLds lstm_bwd_lds(int T, int H, bool scan, bool fused) {
  LstmBwdLds L{};
  const size_t G4 = 4 * (size_t)H, np = (size_t)((T - 1) / 2);
  L.cf = 0; L.h = L.cf + (size_t)T * 6 * H; L.d = L.h + (size_t)T * H;
  if (!fused) {
    L.dgs = L.d + (size_t)T * H; L.junk = L.dgs + T * G4; L.gpart = L.junk + 64;
    L.total = L.gpart + lstm_gpart_floats(H);
    if (scan) {
      L.M = L.total; L.y = L.M + (size_t)T * 64; L.W = L.y + (size_t)T * 8; L.N = L.W + 64; L.v = L.N + np * 64;
      L.total = L.v + np * 8;
    }
    return L;
  }
  L.y = L.d + (size_t)T * H; L.W = L.y + (size_t)T * 8; L.junk = L.W + 64;
  const size_t u = L.junk + 64;
  L.N = u; L.v = L.N + np * 64;
  L.dgs = u; L.gpart = L.dgs + T * G4;
  const size_t a = np * 72, b = T * G4 + lstm_gpart_floats(H);
  L.total = u + (a > b ? a : b);
  L.M = 0;                                        // global (UpdJob::mscr)
  return L;
}

// FUSED (the tail launch k_lstm_tail): the incoming gradient dpp is produced by the period blocks
// of the same launch. Single layer of width 4 (the dense-state path): the block waits for their
// count (J.tail_ctr) only right before the pair maps, after the pre-pass and the step matrices;
// the step matrices go to global scratch (LDS map above). Any other shape (H = 8, stacked layers)
// runs k_lstm_bwd's serial chain in k_lstm_bwd's LDS map and waits after the top layer's pre-pass.
// The layer-0 W_ih gradient (k_wgrad's sum, same order) is handed to the launch's helper blocks.
template <int HM, bool FUSED>
DLAP_DEV void lstm_bwd_body(const UpdJob& J, const ModelDesc* __restrict__ md, int scan, float* sm, bool tsm) {
  if (md->nrnn == 0) return;
  const int T = J.T, M = md->M, H = md->H, G4 = 4 * H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool drop = J.dropout > 0.f;
  const uint32_t thr = (uint32_t)(J.dropout * 16777216.f + 0.5f);
  const float scale = drop ? 1.f / (1.f - J.dropout) : 1.f;
  const uint32_t step = (uint32_t)*gp(J.drop_step);
  const auto params = gp(J.params);
  const auto grads = gp(J.grads);
  RNN_TS(8, tsm);
  // the dense-state BPTT at H = 4: k_lstm_bwd with `scan`, the fused tail always (every layer; the
  // same path and summation order as k_lstm_bwd, so both give the same bits)
  const bool dense = HM == 4 && H == 4 && (FUSED || scan != 0);
  const LstmBwdLds LL = lstm_bwd_lds(T, H, dense && !FUSED, FUSED && dense);
  float* s_cf = sm + LL.cf;                    // [T][6][H] BPTT coefficients (pre-pass)
  float* s_h = sm + LL.h;                      // [T][H]  layer outputs
  float* s_d = sm + LL.d;                      // [T][H]  incoming gradient
  float* dgs = sm + LL.dgs;                    // [T][4H] gate pre-activation gradients
  float* junk0 = sm + LL.junk;                 // 64 junk slots (stores of non-owner lanes)
  __shared__ int s_bad;                        // FUSED: the wait for dpp gave up
  if (FUSED && threadIdx.x == 0) s_bad = 0;
  if (FUSED) __syncthreads();
  // FUSED: the incoming gradient: every period block of this launch has published dpp[t]
  // (write-through stores, drained, then one agent-scope add each). Wave 0 polls the count
  // (relaxed, s_sleep between polls, bounded), ONE agent acquire; false: gave up (block-uniform)
  auto wait_dpp = [&]() -> bool {
    if (threadIdx.x < 64) {
      const int* ctr = J.tail_ctr;
      int v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      unsigned spins = 0;
      while (v < T) {
        if (spins++ >= J.spin_limit) {         // never on a resident grid: poison the model
          if (threadIdx.x == 0) { atomicAdd(const_cast<int*>(J.prog) + 1, 1); s_bad = 1; }
          break;
        }
        __builtin_amdgcn_s_sleep(2);
        v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    return s_bad == 0;
  };
  for (int l = md->nrnn - 1; l >= 0; --l) {
    const auto dout = l == md->nrnn - 1 ? gp(J.dpp) : gp(J.dx);
    // (FUSED: the top layer's incoming gradient is loaded after the wait)
    const bool late_d = FUSED && l == md->nrnn - 1;
    const auto sgg = gp(J.sg) + (size_t)l * T * G4;
    const auto scg = gp(J.sc) + (size_t)l * T * H;
    const auto shg = gp(J.sh) + (size_t)l * T * H;
    // W_hh of the layer for the dense-state path's step matrices: loaded with the pre-pass
    // (its latency hides behind the pre-pass loads), stored after the pre-pass barrier
    const float whh_l = threadIdx.x < 64 ? params[md->lstm_w_hh[l] + (threadIdx.x < 4 * H * H ? threadIdx.x : 0)] : 0.f;
    __syncthreads();
    // parallel pre-pass: everything of the backward step that does not depend on dh_next.
    // PU elements per thread with every global load issued before the first use (one memory
    // round trip instead of one per element)
    constexpr int PU = 4;
    for (int i0 = threadIdx.x; i0 < T * H; i0 += 256 * PU) {
      float gi[PU], gf[PU], gg[PU], go[PU], c[PU], cp[PU], hv[PU], dv[PU];
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const int i = min(i0 + 256 * u, T * H - 1);
        const int t = i / H, k = i - t * H;
        gi[u] = sgg[(size_t)t * G4 + k];
        gf[u] = sgg[(size_t)t * G4 + H + k];
        gg[u] = sgg[(size_t)t * G4 + 2 * H + k];
        go[u] = sgg[(size_t)t * G4 + 3 * H + k];
        c[u] = scg[i];
        cp[u] = t > 0 ? scg[i - H] : (J.c0 ? gp(J.c0)[l * H + k] : 0.f);
        hv[u] = shg[i];
        dv[u] = late_d ? 0.f : dout[i];
      }
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const int i = i0 + 256 * u;
        if (i >= T * H) break;
        const int t = i / H, k = i - t * H;
        const float tc = ftanh(c[u]);
        float* q = s_cf + t * LSTM_NCOEF * H + k;
        q[0 * H] = go[u] * (1.f - tc * tc);
        q[1 * H] = gg[u] * gi[u] * (1.f - gi[u]);
        q[2 * H] = cp[u] * gf[u] * (1.f - gf[u]);
        q[3 * H] = gi[u] * (1.f - gg[u] * gg[u]);
        q[4 * H] = tc * go[u] * (1.f - go[u]);
        q[5 * H] = gf[u];
        s_h[i] = hv[u];
        if (!late_d) s_d[i] = dv[u];
      }
    }
    __syncthreads();
    if (l == 0) RNN_TS(9, tsm);
    if (wave == 0) __builtin_amdgcn_s_setprio(3);     // serial chain: see k_lstm_gls
    if (late_d && !dense) {
      if (!wait_dpp()) return;
      for (int i = threadIdx.x; i < T * H; i += 256) s_d[i] = dout[i];
      __syncthreads();
    }
    if (dense) {
      // ---- dense-state BPTT (header comment): step matrices, chain on wave 0, gate gradients
      float* s_M = FUSED ? gp(J.mscr) : sm + LL.M;   // [T][64] step matrices
      float* s_y = sm + LL.y;
      float* s_W = sm + LL.W;
      float* s_N = sm + LL.N;                         // [(T-1)/2][64] pair maps N_t
      float* s_v = sm + LL.v;                         // [(T-1)/2][8]  pair offsets v_t
      if (threadIdx.x < 64) s_W[threadIdx.x] = whh_l;
      __syncthreads();
      // one thread per (t, row i): the step's 24 coefficients as six 16-byte reads, the row's
      // W_hh column in registers, two 16-byte stores
      {
        const int i = threadIdx.x & 7;
        float wc[16];                                  // wc[r] = W_hh[r][i] (rows r = 4q + k)
#pragma unroll
        for (int r = 0; r < 16; ++r) wc[r] = s_W[r * 4 + (i & 3)];
        // SU steps per pass with every coefficient read issued before the first store (the stores
        // may alias the reads as far as the compiler knows: one LDS round trip per pass, not per step)
        constexpr int SU = 4;
        for (int t0 = threadIdx.x >> 3; t0 < T; t0 += 32 * SU) {
          f32x4 A[SU], Bi[SU], Bf[SU], Bg[SU], Bo[SU], F[SU];
#pragma unroll
          for (int u = 0; u < SU; ++u) {
            const int t = min(t0 + 32 * u, T - 1);
            const f32x4* q4 = reinterpret_cast<const f32x4*>(s_cf + t * (LSTM_NCOEF * 4));
            A[u] = q4[0]; Bi[u] = q4[1]; Bf[u] = q4[2]; Bg[u] = q4[3]; Bo[u] = q4[4]; F[u] = q4[5];
          }
#pragma unroll
          for (int u = 0; u < SU; ++u) {
            const int t = t0 + 32 * u;
            if (t >= T) break;
            f32x4 lo, hi;
            if (i < 4) {                               // row i of dh_next' (= unit j = i)
#pragma unroll
              for (int k = 0; k < 4; ++k) {
                const float pc = wc[k] * Bi[u][k] + wc[4 + k] * Bf[u][k] + wc[8 + k] * Bg[u][k];
                lo[k] = fmaf(pc, A[u][k], wc[12 + k] * Bo[u][k]);
                hi[k] = pc;
              }
            } else {                                   // row of dc_next' (unit k = i - 4)
              const int k = i - 4;
#pragma unroll
              for (int c = 0; c < 4; ++c) {
                lo[c] = c == k ? F[u][c] * A[u][c] : 0.f;
                hi[c] = c == k ? F[u][c] : 0.f;
              }
            }
            f32x4* dst = reinterpret_cast<f32x4*>(s_M + t * 64 + 8 * i);
            dst[0] = lo;
            dst[1] = hi;
          }
        }
      }
      // pair maps: the chain advances two steps per link, y_t = N_t y_{t+2} + v_t for the chain
      // points t = T-1-2p (p = 1 .. np), N_t = M_{t+1} M_{t+2}, v_t = M_{t+1} (dout_{t+1}, 0) +
      // (dout_t, 0); one thread per (link, row), fixed summation order. The maps N_t need only
      // the step matrices, so they are formed before the wait for the incoming gradient (fused
      // tail: while the period blocks publish it); the offsets v_t after it.
      __syncthreads();
      const int npair = (T - 1) / 2;
      constexpr int PU2 = 2;                           // links per pass, reads hoisted (as above)
      for (int task0 = threadIdx.x; task0 < npair * 8; task0 += 256 * PU2) {
        f32x4 a0[PU2], a1[PU2], mb[PU2][16];
#pragma unroll
        for (int u = 0; u < PU2; ++u) {
          const int task = min(task0 + 256 * u, npair * 8 - 1);
          const int p = 1 + (task >> 3), i = task & 7, t = T - 1 - 2 * p;
          const f32x4* ra = reinterpret_cast<const f32x4*>(s_M + (t + 1) * 64 + 8 * i);
          a0[u] = ra[0];
          a1[u] = ra[1];
          const f32x4* m4 = reinterpret_cast<const f32x4*>(s_M + (t + 2) * 64);
#pragma unroll
          for (int k = 0; k < 16; ++k) mb[u][k] = m4[k];
        }
#pragma unroll
        for (int u = 0; u < PU2; ++u) {
          const int task = task0 + 256 * u;
          if (task >= npair * 8) break;
          const int p = 1 + (task >> 3), i = task & 7;
          const float a[8] = {a0[u][0], a0[u][1], a0[u][2], a0[u][3], a1[u][0], a1[u][1], a1[u][2], a1[u][3]};
          f32x4 lo = zero4(), hi = zero4();
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            lo = lo + a[k] * mb[u][2 * k];
            hi = hi + a[k] * mb[u][2 * k + 1];
          }
          f32x4* dn = reinterpret_cast<f32x4*>(s_N + (p - 1) * 64 + 8 * i);
          dn[0] = lo;
          dn[1] = hi;
        }
      }
      if (FUSED && late_d) {
        if (!wait_dpp()) return;                     // block-uniform; nothing written
        for (int i = threadIdx.x; i < T * H; i += 256) s_d[i] = dout[i];
        RNN_TS(16, tsm);
      }
      __syncthreads();
      __syncthreads();
      for (int task0 = threadIdx.x; task0 < npair * 8; task0 += 256 * PU2) {
        f32x4 a0[PU2], du[PU2];
        float dt[PU2];
#pragma unroll
        for (int u = 0; u < PU2; ++u) {
          const int task = min(task0 + 256 * u, npair * 8 - 1);
          const int p = 1 + (task >> 3), i = task & 7, t = T - 1 - 2 * p;
          a0[u] = reinterpret_cast<const f32x4*>(s_M + (t + 1) * 64 + 8 * i)[0];
          du[u] = *reinterpret_cast<const f32x4*>(s_d + (t + 1) * 4);
          dt[u] = s_d[t * 4 + (i & 3)];
        }
#pragma unroll
        for (int u = 0; u < PU2; ++u) {
          const int task = task0 + 256 * u;
          if (task >= npair * 8) break;
          const int p = 1 + (task >> 3), i = task & 7;
          float v = a0[u][0] * du[u][0] + a0[u][1] * du[u][1] + a0[u][2] * du[u][2] + a0[u][3] * du[u][3];
          if (i < 4) v += dt[u];
          s_v[(p - 1) * 8 + i] = v;
        }
      }
      __syncthreads();
      if (l == 0) RNN_TS(13, tsm);
      if (wave == 0) {
        const int i = lane >> 3, j = lane & 7;
        const int offA = 8 * i + j, offB = 8 * j + i;
        // per-link state records without exec-mask changes: the owner lanes of a layout (j == 0
        // in R, i == 0 in C) store y_t, the others write a junk slot (the old path's)
        float* junk = junk0;
        float* dstR = j == 0 ? s_y + i : junk + lane;
        float* dstC = i == 0 ? s_y + j : junk + lane;
        const int strR = j == 0 ? 16 : 0, strC = i == 0 ? 16 : 0;     // two steps per link
        // y_{T-1} = (dout_{T-1}, 0) in the C layout
        float y = j < 4 ? s_d[(T - 1) * 4 + j] : 0.f;
        if (i == 0) s_y[(T - 1) * 8 + j] = y;
        float* yR = dstR + (T - 1) * (j == 0 ? 8 : 0);   // record of link p at yR - p * strR
        float* yC = dstC + (T - 1) * (i == 0 ? 8 : 0);
        // links in blocks of U (even: every block starts from the C layout), the next block's
        // operands loaded a whole block ahead
        constexpr int U = 8;
        float mA[U], uA[U], mB[U], uB[U];
        auto load_block = [&](int p0, float (&m)[U], float (&u)[U]) {
#pragma unroll
          for (int k = 0; k < U; ++k) {
            const int pp = min(p0 + k, npair) - 1;
            const bool ev = (k & 1) == 0;
            m[k] = s_N[pp * 64 + (ev ? offA : offB)];
            u[k] = s_v[pp * 8 + (ev ? i : j)];
          }
        };
        auto run_block = [&](int p0, const float (&m)[U], const float (&u)[U]) {
#pragma unroll
          for (int k = 0; k < U; ++k) {
            const int pp = p0 + k;
            const float pr = rmul(m[k], y);
            if ((k & 1) == 0) {
              y = red8_j(pr) + u[k];
              yR[-pp * strR] = y;
            } else {
              y = red8_i(pr) + u[k];
              yC[-pp * strC] = y;
            }
          }
        };
        const int nfull = npair / U;
        int p = 1;
        if (nfull > 0) load_block(p, mA, uA);
        for (int b = 0; b < nfull; b += 2) {
          if (b + 1 < nfull) load_block(p + U, mB, uB);
          run_block(p, mA, uA);
          p += U;
          if (b + 1 < nfull) {
            if (b + 2 < nfull) load_block(p + U, mA, uA);
            run_block(p, mB, uB);
            p += U;
          }
        }
        bool cl = true;                                // C layout after an even number of links
        for (; p <= npair; ++p) {
          const float m = s_N[(p - 1) * 64 + (cl ? offA : offB)];
          const float u = s_v[(p - 1) * 8 + (cl ? i : j)];
          const float pr = rmul(m, y);
          y = (cl ? red8_j(pr) : red8_i(pr)) + u;
          if (cl) yR[-p * strR] = y;
          else yC[-p * strC] = y;
          cl = !cl;
        }
      }
      __syncthreads();
      // the steps between chain points, in parallel: y_t = M_{t+1} y_{t+1} + (dout_t, 0)
      for (int task = threadIdx.x; task < (T / 2) * 8; task += 256) {
        const int t = T - 2 - 2 * (task >> 3), i = task & 7;
        const f32x4* ra = reinterpret_cast<const f32x4*>(s_M + (t + 1) * 64 + 8 * i);
        const f32x4* yb = reinterpret_cast<const f32x4*>(s_y + (t + 1) * 8);
        const f32x4 a0 = ra[0], a1 = ra[1], y0 = yb[0], y1 = yb[1];
        float v = a0[0] * y0[0] + a0[1] * y0[1] + a0[2] * y0[2] + a0[3] * y0[3] +
                  (a1[0] * y1[0] + a1[1] * y1[1] + a1[2] * y1[2] + a1[3] * y1[3]);
        if (i < 4) v += s_d[t * 4 + i];
        s_y[t * 8 + i] = v;
      }
      __syncthreads();
      // dL/d(initial state): the state leaving step 0, M_0 y_0
      if (J.dh0 && threadIdx.x < 8) {
        const int i = threadIdx.x;
        float v = 0.f;
        for (int k = 0; k < 8; ++k) v += s_M[8 * i + k] * s_y[k];
        if (i < 4) gp(J.dh0)[l * 4 + i] = v;
        else gp(J.dc0)[l * 4 + (i - 4)] = v;
      }
      __syncthreads();
      if (l == 0) RNN_TS(15, tsm);
      // gate gradients from the recorded states: dh = y_h, dc = A dh + y_c
      for (int idx = threadIdx.x; idx < T * 4; idx += 256) {
        const int t = idx >> 2, k = idx & 3;
        const float* q = s_cf + t * (LSTM_NCOEF * 4);
        const float dh = s_y[t * 8 + k];
        const float dc = fmaf(dh, q[k], s_y[t * 8 + 4 + k]);
        float* d = dgs + t * 16 + k;
        d[0] = dc * q[4 + k];
        d[4] = dc * q[8 + k];
        d[8] = dc * q[12 + k];
        d[12] = dh * q[16 + k];
      }
    } else if (wave == 0 && HM == 4 && H == 4) {
      // Gate-per-lane BPTT (H = 4): lane L (mod 16) owns gate row L = 4q + k and keeps the
      // recurrent state of unit k replicated, so d_L = (q == 3 ? dh : dc) * coef is lane-local
      // and dh_next_j = sum_L W_hh[L][j] d_L is ONE reduce-scatter over the 16 lanes: two DPP
      // quad exchanges (xor 1: 4 -> 2 values, xor 2: 2 -> 1) and two row rotations, after which
      // lane L holds the sum for j = L & 3 = its own unit. Branch-free; rows 1..3 of the wave
      // duplicate row 0 and store to a junk slot.
      const int L16 = lane & 15, kq = L16 >> 2, ku = L16 & 3;
      const bool b0 = (lane & 1) != 0, b1 = (lane & 2) != 0, isO = kq == 3;
      const auto Whh = params + md->lstm_w_hh[l];
      float w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = Whh[L16 * 4 + j];
      float* junk = junk0;
      float* ddst = lane < 16 ? dgs + L16 : junk + lane;
      const int dstride = lane < 16 ? 16 : 0;
      const int ci = (1 + kq) * 4 + ku;
      float dh_next = 0.f, dc_next = 0.f;
      auto fetch = [&](int t, float (&v)[4]) {
        const float* q = s_cf + t * (LSTM_NCOEF * 4);
        v[0] = q[ku]; v[1] = q[20 + ku]; v[2] = q[ci]; v[3] = s_d[t * 4 + ku];
      };
      auto step = [&](int t, const float (&v)[4]) {
        const float dh = v[3] + dh_next;
        const float dc = dh * v[0] + dc_next;
        dc_next = dc * v[1];
        const float d = (isO ? dh : dc) * v[2];
        ddst[t * dstride] = d;
        const float p0 = w[0] * d, p1 = w[1] * d, p2 = w[2] * d, p3 = w[3] * d;
        const float a0 = b0 ? p1 : p0, s0 = b0 ? p0 : p1;
        const float a1 = b0 ? p3 : p2, s1 = b0 ? p2 : p3;
        const float n0 = a0 + dppf<0xB1>(s0);             // quad_perm [1,0,3,2]
        const float n1 = a1 + dppf<0xB1>(s1);
        const float a = b1 ? n1 : n0, sx = b1 ? n0 : n1;
        float r = a + dppf<0x4E>(sx);                      // quad_perm [2,3,0,1]
        r += dppf<0x124>(r);                               // row_ror:4
        r += dppf<0x128>(r);                               // row_ror:8
        dh_next = r;
      };
      constexpr int U = 8;
      const int nfull = T / U;
      int t = T - 1;
      for (; t >= nfull * U; --t) {
        float v[4];
        fetch(t, v);
        step(t, v);
      }
      float A[U][4], B[U][4];
      auto load_block = [&](int t0, float (&buf)[U][4]) {
#pragma unroll
        for (int u = 0; u < U; ++u) fetch(t0 - u, buf[u]);
      };
      if (nfull > 0) load_block(t, A);
      for (int b = 0; b < nfull; b += 2) {
        if (b + 1 < nfull) load_block(t - U, B);
#pragma unroll
        for (int u = 0; u < U; ++u) step(t - u, A[u]);
        t -= U;
        if (b + 1 < nfull) {
          if (b + 2 < nfull) load_block(t - U, A);
#pragma unroll
          for (int u = 0; u < U; ++u) step(t - u, B[u]);
          t -= U;
        }
      }
      // dL/d(initial state) of the layer: the gradients carried past t = 0
      if (J.dh0 && lane < 4) { gp(J.dh0)[l * 4 + lane] = dh_next; gp(J.dc0)[l * 4 + lane] = dc_next; }
    } else if (wave == 0) {
      const int k = lane < H ? lane : 0;
      const bool act = lane < H;
      const auto Whh = params + md->lstm_w_hh[l];
      float wt[4][HM];            // wt[q][j] = W_hh[q*H + j][k] (0 for padded j)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < HM; ++j) {
          const float w = Whh[(q * H + (j < H ? j : 0)) * H + k];
          wt[q][j] = j < H ? w : 0.f;
        }
      float dh_next = 0.f, dc_next = 0.f;
      auto fetch = [&](int t, float (&v)[7]) {
        const float* q = s_cf + t * LSTM_NCOEF * H + k;
#pragma unroll
        for (int e = 0; e < LSTM_NCOEF; ++e) v[e] = q[e * H];
        v[6] = act ? s_d[t * H + k] : 0.f;
      };
      auto step = [&](int t, const float (&v)[7]) {
        const float dh = v[6] + dh_next;
        const float dc = dh * v[0] + dc_next;
        float d[4];
        d[0] = dc * v[1];
        d[1] = dc * v[2];
        d[2] = dc * v[3];
        d[3] = dh * v[4];
        dc_next = dc * v[5];
        if (act) {
#pragma unroll
          for (int q = 0; q < 4; ++q) dgs[t * G4 + q * H + k] = d[q];
        }
        const float s = (bcast_dot<HM>(wt[0], d[0]) + bcast_dot<HM>(wt[1], d[1])) +
                        (bcast_dot<HM>(wt[2], d[2]) + bcast_dot<HM>(wt[3], d[3]));
        dh_next = act ? s : 0.f;
      };
      // blocks of U steps; the next block's LDS operands are loaded a whole block ahead
      constexpr int U = 8;
      const int nfull = T / U;
      int t = T - 1;
      for (; t >= nfull * U; --t) {              // top remainder, one at a time
        float v[7];
        fetch(t, v);
        step(t, v);
      }
      float A[U][7], B[U][7];
      auto load_block = [&](int t0, float (&buf)[U][7]) {
#pragma unroll
        for (int u = 0; u < U; ++u) fetch(t0 - u, buf[u]);
      };
      if (nfull > 0) load_block(t, A);
      for (int b = 0; b < nfull; b += 2) {
        if (b + 1 < nfull) load_block(t - U, B);
#pragma unroll
        for (int u = 0; u < U; ++u) step(t - u, A[u]);
        t -= U;
        if (b + 1 < nfull) {
          if (b + 2 < nfull) load_block(t - U, A);
#pragma unroll
          for (int u = 0; u < U; ++u) step(t - u, B[u]);
          t -= U;
        }
      }
      if (J.dh0 && act) { gp(J.dh0)[l * H + k] = dh_next; gp(J.dc0)[l * H + k] = dc_next; }
    }
    __syncthreads();
    if (l == 0) RNN_TS(10, tsm);
    if (l == 0 && !FUSED) {
      const auto dg = gp(J.dg);
      for (int i = threadIdx.x; i < T * G4; i += 256) dg[i] = dgs[i];   // for k_wgrad
    }
    if (l == 0 && FUSED) {
      // hand the gate gradients to the W_ih helper blocks of the launch (R1: write-through stores,
      // every wave drains, barrier, one flag store); they run k_wgrad's sums while this block forms
      // the W_hh / bias gradients
      const auto dg = gp(J.dg);
      for (int i = threadIdx.x; i < T * G4; i += 256)
        __hip_atomic_store(dg + i, dgs[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_store(J.tail_ctr + TAIL_FLAG, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // W_hh [4H][H] and the biases: (gate, column) outputs x S time segments over the 256
    // threads (S = 3 at H = 4: 240 of them busy instead of 80), segment partials summed in
    // segment order from LDS (fixed order: deterministic)
    const int in_dim = l == 0 ? M : H;
    const uint32_t key_below = l > 0 ? dropout_key(J.seed, step, 32 + (l - 1)) : 0u;
    const auto hb = gp(J.sh) + (size_t)(l > 0 ? l - 1 : 0) * T * H;
    const int ncol = H + 1 + (l > 0 ? H : 0);
    const int nout = G4 * ncol;
    const int S = max(1, min(LSTM_GSEG, 256 / max(nout, 1)));
    float* gpart = sm + LL.gpart;                     // [S][nout] (after the gate gradients)
    if (HM == 4 && H == 4) {
      // H = 4: [ncol x 16 gates] = sum_t x[t][col] dG[t][g] on v_mfma_f32_16x16x4f32 (exact
      // fp32 products) -- x = (h_{t-1} (the initial state at t = 0), 1 for the biases, the layer
      // input of a deeper layer). Wave w takes the 4-period k-steps w, w + 4, ...; the four
      // partial tiles are summed in wave order (fixed order: deterministic).
      //   A lane l -> x[t0 + (l >> 4)][col = l & 15],  B lane l -> dG[t0 + (l >> 4)][g = l & 15]
      //   C lane l, r -> (col = 4 (l >> 4) + r, g = l & 15)
      const int lc = lane & 15, lk = lane >> 4;
      const float h0c = (lc < 4 && J.h0) ? gp(J.h0)[l * 4 + lc] : 0.f;
      f32x4 acc = zero4();
      for (int kb = wave; kb * 4 < T; kb += 4) {
        const int t = kb * 4 + lk;
        const bool ok = t < T;
        const int tc = ok ? t : T - 1;
        float a = 0.f;
        if (lc < 4) a = tc > 0 ? s_h[(tc - 1) * 4 + lc] : h0c;
        else if (lc == 4) a = 1.f;
        else if (lc < 9 && l > 0) {
          const int m = lc - 5;
          a = hb[(size_t)tc * 4 + m];
          if (drop) a = dropout_keep(key_below, (uint32_t)tc, (uint32_t)m, thr) ? a * scale : 0.f;
        }
        const float b = dgs[tc * 16 + lc];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ok ? a : 0.f, ok ? b : 0.f, acc, 0, 0, 0);
      }
      *reinterpret_cast<f32x4*>(gpart + wave * 256 + lane * 4) = acc;
      __syncthreads();
      for (int o = threadIdx.x; o < ncol * 16; o += 256) {
        const int col = o >> 4, g = o & 15;
        const int li = 16 * (col >> 2) + g, r = col & 3;
        const float v = ((gpart[li * 4 + r] + gpart[256 + li * 4 + r]) + gpart[512 + li * 4 + r]) + gpart[768 + li * 4 + r];
        if (col < 4) st_wt(grads + md->lstm_w_hh[l] + g * 4 + col, v);
        else if (col == 4) { st_wt(grads + md->lstm_b_ih[l] + g, v); st_wt(grads + md->lstm_b_hh[l] + g, v); }
        else st_wt(grads + md->lstm_w_ih[l] + g * in_dim + (col - 5), v);
      }
      __syncthreads();
    } else
    for (int idx0 = 0; idx0 < nout; idx0 += 256 / S) {
      const int lt = (int)threadIdx.x % (256 / S), seg = (int)threadIdx.x / (256 / S);
      const int idx = idx0 + lt;
      float acc = 0.f;
      if (idx < nout && seg < S) {
        const int g = idx % G4, col = idx / G4;
        const int ta = (T * seg) / S, tb = (T * (seg + 1)) / S;
        if (col < H) {
#pragma unroll 4
          for (int t = max(ta, 1); t < tb; ++t) acc += dgs[t * G4 + g] * s_h[(t - 1) * H + col];
          if (ta == 0 && J.h0) acc += dgs[g] * gp(J.h0)[l * H + col];     // h_{-1} = initial state
        } else if (col == H) {
#pragma unroll 4
          for (int t = ta; t < tb; ++t) acc += dgs[t * G4 + g];
        } else {
          const int m = col - H - 1;     // W_ih of layer l > 0 (input = dropout(h_{l-1}))
          for (int t = ta; t < tb; ++t) {
            float x = hb[(size_t)t * H + m];
            if (drop) x = dropout_keep(key_below, (uint32_t)t, (uint32_t)m, thr) ? x * scale : 0.f;
            acc += dgs[t * G4 + g] * x;
          }
        }
        gpart[seg * nout + idx] = acc;
      }
      __syncthreads();
      if ((int)threadIdx.x < 256 / S && idx0 + (int)threadIdx.x < nout) {
        const int o = idx0 + threadIdx.x, g = o % G4, col = o / G4;
        float v = 0.f;
        for (int q = 0; q < S; ++q) v += gpart[q * nout + o];
        if (col < H) st_wt(grads + md->lstm_w_hh[l] + g * H + col, v);
        else if (col == H) { st_wt(grads + md->lstm_b_ih[l] + g, v); st_wt(grads + md->lstm_b_hh[l] + g, v); }
        else st_wt(grads + md->lstm_w_ih[l] + g * in_dim + (col - H - 1), v);
      }
      __syncthreads();
    }
    if (l > 0) {
      const auto Wih = params + md->lstm_w_ih[l];
      const auto dx = gp(J.dx);
      for (int idx = threadIdx.x; idx < T * H; idx += 256) {
        const int t = idx / H, m = idx - t * H;
        float s = 0.f;
        for (int g = 0; g < G4; ++g) s += Wih[g * H + m] * dgs[t * G4 + g];
        if (drop) s = dropout_keep(key_below, (uint32_t)t, (uint32_t)m, thr) ? s * scale : 0.f;
        dx[idx] = s;
      }
      __threadfence_block();
    }
    // (fused tail, stacked layers: the next layer rewrites the global step-matrix scratch this one
    // read -- drop this CU's cached copies of it; the layer input gradient dx is read back, too)
    if (FUSED && l > 0) {
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
    }
  }
  __syncthreads();
  if constexpr (FUSED) {
    // every period block has added to the count (the wait saw all T): rearm it for the next launch
    if (threadIdx.x == 0) __hip_atomic_store(J.tail_ctr + TAIL_CNT, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  RNN_TS(11, tsm);
}

template <int HM>
__global__ __launch_bounds__(256) void k_lstm_bwd(const UpdJob* __restrict__ jobs,
                                                  const ModelDesc* __restrict__ md, int scan) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  lstm_bwd_body<HM, false>(jobs[blockIdx.x], md, scan, sm, blockIdx.x == 0);
}

// --------------------------------------------------------------------------- k_wgrad ---
// out[g][col] = sum_t dG[t][g] * x[t][col] (x = macro, or 1 for the bias column col = M) for the
// layer-0 LSTM input weights (phases 1/3, dG = gate gradients) or the moment layer-0 macro
// columns + bias (phase 2, dG = per-period sums of the pre-activation gradient).
// fp32 MFMA (v_mfma_f32_16x16x4f32: exact fp32 products): C^T[col][g] = sum_t A[col][t] B[t][g],
//   A lane l -> x[t = t0 + (l>>4)][col = c0 + (l&15)],  B lane l -> dG[t0 + (l>>4)][g0 + (l&15)],
//   C lane l -> (col = c0 + 4(l>>4) + r, g = g0 + (l&15)).
// grid (ceil((M+1)/16), models), 4 waves split the time axis, every operand of a wave's 16
// k-steps is requested before the first MFMA; the 4 partial tiles are summed in LDS in wave order.
// done: the fused tail's helper form -- after every wave has read its operands, one lane counts
// the block on *done (agent scope); the last of ndone rearms the hand-off words for the next launch
// before_dg: called by every thread once, after the first k-chunk's macro operands are requested
// and before any gate-gradient load (the fused tail's helpers wait for the hand-off there, with
// their constant operands already in flight); returns false to abandon the block (block-uniform).
struct NoWait { DLAP_DEV bool operator()() const { return true; } };
// red: [4][GT][64] f32x4 of LDS (the fused tail passes its dynamic LDS)
template <int GT, typename BeforeDG = NoWait>
DLAP_DEV void wgrad_block(const UpdJob& J, const ModelDesc* __restrict__ md, int phase, int cblk, f32x4* red_,
                          int* done = nullptr, int ndone = 0, BeforeDG before_dg = NoWait{}) {
  auto red = reinterpret_cast<f32x4 (*)[GT][64]>(red_);
  const int T = J.T, M = md->M;
  const bool mom = phase == 2;
  const int G = mom ? md->m[0].out : 4 * md->H;
  const int ldG = mom ? 64 : G;
  const auto dG = gp(mom ? J.dab : J.dg);
  const auto X = gp(J.macro);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, n = lane & 15, kq = lane >> 4;
  const int c0 = cblk * 16, col = c0 + n;
  const int ta = (T * wave) / 4, tb = (T * (wave + 1)) / 4;
  f32x4 acc[GT];
#pragma unroll
  for (int gt = 0; gt < GT; ++gt) acc[gt] = zero4();
  constexpr int KC = 16;
  float a[KC], b[KC][GT];
  auto load_x = [&](int t0) {
#pragma unroll
    for (int s = 0; s < KC; ++s) {
      const int t = t0 + 4 * s + kq;
      const bool ok = t < tb;
      const int tc = ok ? t : ta;
      const float x = X[(size_t)tc * M + (col < M ? col : 0)];
      a[s] = ok ? (col < M ? x : (col == M ? 1.f : 0.f)) : 0.f;
    }
  };
  load_x(ta);                                   // (harmless when this wave's range is empty)
  if (!before_dg()) return;
  for (int t0 = ta; t0 < tb; t0 += 4 * KC) {
    if (t0 != ta) load_x(t0);
#pragma unroll
    for (int s = 0; s < KC; ++s) {
      const int t = t0 + 4 * s + kq;
      const bool ok = t < tb;
      const int tc = ok ? t : ta;
#pragma unroll
      for (int gt = 0; gt < GT; ++gt) {
        const int g = gt * 16 + n;
        const float v = dG[(size_t)tc * ldG + (g < G ? g : 0)];
        b[s][gt] = ok && g < G ? v : 0.f;
      }
    }
#pragma unroll
    for (int s = 0; s < KC; ++s)
#pragma unroll
      for (int gt = 0; gt < GT; ++gt) acc[gt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s][gt], acc[gt], 0, 0, 0);
  }
#pragma unroll
  for (int gt = 0; gt < GT; ++gt) red[wave][gt][lane] = acc[gt];
  __syncthreads();
  if (done && threadIdx.x == 0) {
    const int prev = __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == ndone - 1) {               // every helper has read dg: rearm flag and counter
      __hip_atomic_store(done - (TAIL_DONE - TAIL_FLAG), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (wave != 0) return;
#pragma unroll
  for (int gt = 0; gt < GT; ++gt) {
    const f32x4 v = red[0][gt][lane] + red[1][gt][lane] + red[2][gt][lane] + red[3][gt][lane];
    const int g = gt * 16 + n;
    if (g >= G) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int cc = c0 + 4 * kq + r;
      if (cc > M) continue;
      if (mom) {
        const PackLayer& L0 = md->m[0];
        if (cc < M) st_wt(gp(J.grads) + L0.w_off + (size_t)g * L0.ld + cc, v[r]);
        else st_wt(gp(J.grads) + L0.b_off + g, v[r]);
      } else if (cc < M) {
        st_wt(gp(J.grads) + md->lstm_w_ih[0] + (size_t)g * M + cc, v[r]);
      }
    }
  }
}

template <int GT>
__global__ __launch_bounds__(256) void k_wgrad(const UpdJob* __restrict__ jobs,
                                               const ModelDesc* __restrict__ md, int phase) {
  __shared__ f32x4 red[4][GT][64];
  wgrad_block<GT>(jobs[blockIdx.y], md, phase, blockIdx.x, &red[0][0][0]);
}

// Adam in the fused tail (adam = 2): every block, its own work done, arrives on the model's
// TAIL_ARRIVE count (its write-through stores drained first); the last nadam blocks to arrive
// become the update's Adam blocks (adam_block, the same arithmetic as k_adam's blocks): each
// requests its own operands, then waits -- relaxed polls, bounded, one agent acquire -- until
// every block of the model has arrived and the epoch's evaluation branch has signalled (its
// bookkeeping reads the parameters, the gradient norm and the step counters this update
// writes). Both counts only grow (zeroed with the poison records): launch k of the model's
// tail-Adam launches takes arrivals [k nb, (k + 1) nb) and waits for signal k + 1, so nothing
// is rearmed. The step counters were read by every block before it arrived (step_pre), so
// Adam block 0 advances them as soon as it is released. A wait that gives up poisons the model
// (no update; the host raises). The waiting blocks are the last to arrive, so every block they
// wait for has been dispatched ahead of them or is next in line.
DLAP_DEV void tail_adam(const UpdJob& U, const ModelDesc* __restrict__ md, float lr, int nb, int step_pre,
                        int drop_pre, int phase, bool evgen, bool gen) {
  __shared__ unsigned s_ord;
  __shared__ int s_go;
  __shared__ float red[4];
  // the gradients / job scalars Adam reads are written through (st_wt): each wave drains its
  // stores, then one agent-scope add per block
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    s_ord = __hip_atomic_fetch_add(reinterpret_cast<unsigned*>(U.tail_ctr + (phase == 2 ? TAIL_ARRIVE2 : TAIL_ARRIVE)),
                                   1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const unsigned k = s_ord / (unsigned)nb, ord = s_ord - k * (unsigned)nb;
  const bool tsm = blockIdx.y == 0;
  RNN_TS(18, tsm && ord == (unsigned)nb - 1);                       // the last arrival
  const int nadam = ((phase == 2 ? md->P - md->P_sdf : md->P_sdf) + ADAM_PB - 1) / ADAM_PB;
  const int bx = (int)ord - (nb - nadam);
  if (bx < 0) return;
  auto wait = [&]() -> bool {
    if (threadIdx.x < 64) {
      bool ok = true;
      unsigned spins = 0;
      const unsigned all = (k + 1) * (unsigned)nb;
      const int* arr = U.tail_ctr + (phase == 2 ? TAIL_ARRIVE2 : TAIL_ARRIVE);
      while ((unsigned)__builtin_amdgcn_readfirstlane(__hip_atomic_load(arr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) - all >
             0x7fffffffu) {                                            // (wrap-safe "count < all")
        if (spins++ >= U.spin_limit) { ok = false; break; }
        __builtin_amdgcn_s_sleep(2);
      }
      const int* gen = U.tail_ctr + TAIL_EVGEN;
      while (ok && evgen && (unsigned)__builtin_amdgcn_readfirstlane(__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) -
                           (k + 1) > 0x7fffffffu) {
        if (spins++ >= U.spin_limit) { ok = false; break; }
        __builtin_amdgcn_s_sleep(2);
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (threadIdx.x == 0) {
        if (!ok) atomicAdd(const_cast<int*>(U.prog) + 1, 1);
        s_go = ok && !prog_poisoned(U.prog);
      }
    }
    __syncthreads();
    RNN_TS(19, tsm && bx == 0);                                      // Adam block 0 released
    return s_go != 0;
  };
  adam_block(U, md, phase, lr, bx, nadam, red, wait, step_pre, drop_pre);
  if (gen) {
    // the update is complete once all nadam Adam blocks of the launch are: each counts itself
    // (acq_rel: its stores released, the earlier counts' acquired); the last of the launch advances
    // the model's update generation (release) -- the evaluation graph's k_wait_gen waits for it
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned prev = __hip_atomic_fetch_add(reinterpret_cast<unsigned*>(U.tail_ctr + TAIL_ADONE), 1u,
                                                   __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if ((prev + 1u) % (unsigned)nadam == 0u)
        __hip_atomic_fetch_add(U.tail_ctr + TAIL_UPDGEN, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  RNN_TS(20, tsm && bx == nadam - 1);
}

// Fused backward tail of phases 1 / 3 (one launch instead of k_finalize -> k_lstm_bwd -> k_wgrad
// [-> k_adam]): grid (1 + T + slab blocks + W_ih blocks [+ 1], models). Block 0 runs the LSTM
// backward (lstm_bwd_body<HM, true>: the pre-pass (and, dense-state path, the step matrices)
// first, then it waits for the per-period gradient; every layer of a stacked LSTM); blocks 1 .. T form the per-period sums dpp[t] and publish them; the slab
// blocks sum the weight-gradient slabs; the next (M + 16) / 16 blocks wait for block 0's gate
// gradients and form the layer-0 W_ih gradient (wgrad_block) while block 0 forms W_hh and the
// biases. Every block runs the same arithmetic as the separate kernels, so the results are
// bitwise equal. Blocks 0 and the W_ih blocks wait only for blocks that never wait, and the
// launch (under 400 blocks per model at the bench size) is resident at once on an idle device.
// ljobs (optional): the train split's loss jobs of the step -- one more block per model computes
// its job metrics (k_job_metrics' body; the loss passes finished before this launch), so the
// pipelined epoch needs no fork to the evaluation branch for them.
// adam (tail_adam): the clip + Adam update of the step in the launch's last blocks (2: after
// the evaluation branch's signal; the only mode).
template <int HM>
__global__ __launch_bounds__(256, 2) void k_lstm_tail(const UpdJob* __restrict__ ujobs, const FinJob* __restrict__ fjobs,
                                                   const ModelDesc* __restrict__ md, int slab_stride, int nslab_blocks,
                                                   const LossJob* __restrict__ ljobs, int adam, float lr, int phase) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const UpdJob& U = ujobs[blockIdx.y];
  const FinJob& F = fjobs[blockIdx.y];
  const int b = (int)blockIdx.x - 1;
  const int nwg = (md->M + 1 + 15) / 16;
  const bool mom = phase == 2;
  __shared__ int s_steps[2];          // (adam) the step counters before this launch's update
  if (adam && threadIdx.x == 0) { s_steps[0] = gp(U.adam_step)[mom ? 1 : 0]; s_steps[1] = gp(U.drop_step)[0]; }
  if (b < 0 && mom) {
    // phase 2 (no BPTT): relay the per-period blocks' count to the W_macro helpers -- wait for all
    // T (relaxed polls, bounded, one agent acquire), rearm the count, raise the flag
    __shared__ int bad;
    if (threadIdx.x < 64) {
      const int* ctr = U.tail_ctr + TAIL_CNT;
      unsigned spins = 0;
      bool ok = true;
      while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < U.T) {
        if (spins++ >= U.spin_limit) { ok = false; break; }
        __builtin_amdgcn_s_sleep(2);
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      if (threadIdx.x == 0) {
        bad = ok ? 0 : 1;
        if (!ok) atomicAdd(const_cast<int*>(U.prog) + 1, 1);      // poison: no update, the host raises
        else {
          __hip_atomic_store(U.tail_ctr + TAIL_CNT, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          __hip_atomic_store(U.tail_ctr + TAIL_FLAG, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    __syncthreads();
  } else if (b < 0) {
    lstm_bwd_body<HM, true>(U, md, 1, sm, blockIdx.y == 0);
  } else if (b < U.T) {
    finalize_block(F, md, phase, slab_stride, nslab_blocks + b, U.tail_ctr + TAIL_CNT);
  } else if (b < U.T + nslab_blocks) {
    finalize_block(F, md, phase, slab_stride, b - U.T);
  } else if (b >= U.T + nslab_blocks + nwg) {      // the train split's job metrics
    if (ljobs) job_metrics_body<256>(ljobs[blockIdx.y], sm + DLAP_MAX_T, sm);
  } else {
    // W_ih helper: k_wgrad's block, its macro operands requested first, then the wait for the
    // gate gradients (relaxed poll, one agent acquire, barrier) before their loads
    const int cblk = b - U.T - nslab_blocks;
    __shared__ int bad;
    auto wait_dg = [&]() -> bool {
      if (threadIdx.x < 64) {
        const int* flag = U.tail_ctr + TAIL_FLAG;
        int v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        unsigned spins = 0;
        bool ok = true;
        while (v == 0) {
          if (spins++ >= U.spin_limit) { ok = false; break; }   // block 0 gave up (and poisoned the model)
          __builtin_amdgcn_s_sleep(2);
          v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (threadIdx.x == 0) bad = ok ? 0 : 1;
      }
      __syncthreads();
      return bad == 0;
    };
    f32x4* red = reinterpret_cast<f32x4*>(sm);
    const int G = mom ? md->m[0].out : 4 * md->H;         // gate / moment layer-0 columns
    if (G <= 16) wgrad_block<1>(U, md, phase, cblk, red, U.tail_ctr + TAIL_DONE, nwg, wait_dg);
    else if (G <= 32) wgrad_block<2>(U, md, phase, cblk, red, U.tail_ctr + TAIL_DONE, nwg, wait_dg);
    else wgrad_block<4>(U, md, phase, cblk, red, U.tail_ctr + TAIL_DONE, nwg, wait_dg);
    if (blockIdx.y == 0 && cblk == nwg - 1 && threadIdx.x == 0) g_rnn_ts[17] = wall_clock64();
  }
  if (adam) tail_adam(U, md, lr, gridDim.x, s_steps[0], s_steps[1], phase, adam >= 2, adam == 3);
}

// whether the fused tail applies (phases 1 / 3; LSTM widths up to 8, any depth); its LDS bytes:
// the dense-state map for one layer of width 4, else k_lstm_bwd's
static bool tail_dense(const ModelDesc& mh) { return mh.H == 4; }
size_t lstm_tail_lds_bytes(const ModelDesc& mh, int T) {
  return lstm_bwd_lds(T, mh.H, false, tail_dense(mh)).total * sizeof(float);
}
bool lstm_tail_supported(const ModelDesc& mh, int T) {
  if (mh.nrnn < 1 || mh.H > 8 || mh.M <= 0 || T < 2) return false;
  const char* scan_env = std::getenv("DLAP_LSTM_SCAN");
  if (tail_dense(mh) && scan_env && std::atoi(scan_env) == 0) return false;
  // (+ static LDS) two per CU for the dense map; one per CU otherwise (H = 8: ~100 KB at T = 240).
  // Residency is not required: the only in-kernel waits are on lower-numbered blocks (the LSTM
  // block waits for the period blocks dispatched right after it) or, for Adam, the last arrivals
  const size_t lim = tail_dense(mh) ? 80 * 1024 : 160 * 1024;
  return lstm_tail_lds_bytes(mh, T) + 6400 <= lim;
}
int lstm_tail_words() { return TAIL_WORDS; }
static size_t tail_dyn_lds(const ModelDesc& mh, int T, int phase = 1) {
  // (the metrics block keeps its scratch in the dynamic LDS: DLAP_MAX_T + 4 floats; the W_ih /
  // W_macro helpers their [4][GT][64] f32x4 partial tiles, GT <= 4)
  const size_t small = std::max((size_t)(DLAP_MAX_T + 4) * sizeof(float), (size_t)4 * 4 * 64 * 16);
  return phase == 2 ? small : std::max(lstm_tail_lds_bytes(mh, T), small);
}
bool mom_tail_supported(const ModelDesc& mh, int T) {
  return mh.M > 0 && mh.m[0].out <= 64 && T >= 1;
}
int lstm_tail_capacity(const ModelDesc& mh, int T) {
  const size_t sh = tail_dyn_lds(mh, T);
  int per_cu = 0, dev = 0, ncu = 0;
  if (mh.H <= 4) HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_lstm_tail<4>, 256, sh));
  else HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_lstm_tail<8>, 256, sh));
  HIP_OK(hipGetDevice(&dev));
  HIP_OK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  return per_cu * ncu;
}
void launch_lstm_tail(const UpdJob* ujobs, const FinJob* fjobs, int njobs, const ModelDesc* md, const ModelDesc& mh,
                      int T, int slab_stride, hipStream_t st, const LossJob* ljobs, int adam, float lr, int phase) {
  const int nslab_blocks = (phase == 2 ? mh.ntile_m : mh.ntile_s) * 64 + (SLAB_EXTRA + 63) / 64;
  const int nwg = (mh.M + 1 + 15) / 16;
  const size_t sh = tail_dyn_lds(mh, T, phase);
  const dim3 grid(1 + T + nslab_blocks + nwg + (ljobs ? 1 : 0), njobs);
  if (mh.H <= 4)
    hipLaunchKernelGGL(k_lstm_tail<4>, grid, dim3(256), sh, st, ujobs, fjobs, md, slab_stride, nslab_blocks, ljobs, adam, lr,
                       phase);
  else
    hipLaunchKernelGGL(k_lstm_tail<8>, grid, dim3(256), sh, st, ujobs, fjobs, md, slab_stride, nslab_blocks, ljobs, adam, lr,
                       phase);
  HIP_OK(hipGetLastError());
}

void launch_lstm_bwd(const UpdJob* jobs, int njobs, const ModelDesc* md, const ModelDesc& mh,
                     int T, int phase, hipStream_t st) {
  if (phase != 2 && mh.nrnn > 0) {
    // coef, h, d, dgates, junk, weight-gradient segment partials (+ the dense-state path's
    // step matrices / states when H = 4 and they fit; DLAP_LSTM_SCAN=0 keeps the gate-per-lane
    // chain)
    size_t sh = ((size_t)T * (LSTM_NCOEF + 2 + 4) * mh.H + 64 + lstm_gpart_floats(mh.H)) * sizeof(float);
    if (sh > 160 * 1024) dlap_throw_hip(hipErrorInvalidValue, "lstm_bwd: T*H too large for LDS", __FILE__, __LINE__);
    const char* scan_env = std::getenv("DLAP_LSTM_SCAN");
    const bool scan_on = !(scan_env && std::atoi(scan_env) == 0);
    const size_t sh_scan = sh + lstm_bwd_scan_floats(T) * sizeof(float);
    const int scan = scan_on && mh.H == 4 && T >= 2 && sh_scan <= 160 * 1024 ? 1 : 0;
    if (scan) sh = sh_scan;
    if (mh.H <= 4) hipLaunchKernelGGL((k_lstm_bwd<4>), dim3(njobs), dim3(256), sh, st, jobs, md, scan);
    else if (mh.H <= 8) hipLaunchKernelGGL((k_lstm_bwd<8>), dim3(njobs), dim3(256), sh, st, jobs, md, 0);
    else if (mh.H <= 16) hipLaunchKernelGGL((k_lstm_bwd<16>), dim3(njobs), dim3(256), sh, st, jobs, md, 0);
    else hipLaunchKernelGGL((k_lstm_bwd<32>), dim3(njobs), dim3(256), sh, st, jobs, md, 0);
    HIP_OK(hipGetLastError());
  }
  if (mh.M == 0) return;
  if (phase != 2 && mh.nrnn == 0) return;
  const int G = phase == 2 ? mh.m[0].out : 4 * mh.H;
  dim3 grid((mh.M + 1 + 15) / 16, njobs);
  if (G <= 16) hipLaunchKernelGGL((k_wgrad<1>), grid, dim3(256), 0, st, jobs, md, phase);
  else if (G <= 32) hipLaunchKernelGGL((k_wgrad<2>), grid, dim3(256), 0, st, jobs, md, phase);
  else if (G <= 64) hipLaunchKernelGGL((k_wgrad<4>), grid, dim3(256), 0, st, jobs, md, phase);
  else hipLaunchKernelGGL((k_wgrad<8>), grid, dim3(256), 0, st, jobs, md, phase);
  HIP_OK(hipGetLastError());
}

std::vector<long long> rnn_timestamps() {
  std::vector<long long> v(24);
  HIP_OK(hipMemcpyFromSymbol(v.data(), HIP_SYMBOL(g_rnn_ts), sizeof(long long) * 24));
  return v;
}
