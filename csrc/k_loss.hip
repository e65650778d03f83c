// Fused masked moment-loss kernels.
//
// Reference math (`/root/reference/src/model.py:346-483,565-594`, `src/train.py:29-42,106-153`):
//   w'      = (w - mu_t) m                  mu_t = sum_i w m / max(N_t, 1)   (zero-mean)
//   P_t     = (Nbar / max(N_t,1)) sum_i w' R m                              (weighted loss)
//   E[k,i]  = sum_t h[k,t,i] R m (1 + P_t) / max(T_i, 1)
//   L_cond  = mean_k mean_i E^2,   L_unc = the h == 1 case
// Three passes, each a plain launch (no inter-workgroup hand-offs, fixed-order sums):
//   k_period_fwd  one workgroup per (job, period): mu_t, w', P_t, SDF_t, the L1-normalised
//                 portfolio return (evaluate), residual-loss statistics
//   k_asset       one workgroup per (job, 64 stocks): E, E_unc, dL/dE and partial loss sums;
//                 the 4 waves split the time axis, then reduce in LDS in a fixed order
//                 (A fused 'last block reduces' variant was measured 7x slower: the agent-scope
//                 release fences write back the XCD L2 on every block.)
//   k_period_bwd  one workgroup per (job, period): dL/dSDF_t and the analytic gradient of
//                 the zero-mean normalisation, dL/dw_raw = m c_t (R - mean_t R) (+ residual)
//   k_job_metrics one workgroup per job: scalar losses, Sharpe (unbiased std, 1e-8 guard),
//                 max drawdown (cumprod scan), mean/std of the evaluation returns
#include <cstdlib>

#include "common.h"
#include "loss.h"
#include "loss_dev.h"

// In-kernel timestamps of k_job_metrics, last block (Engine.loss_timestamps, 100 MHz clock):
// [0] start, [1] losses reduced, [2] pass 0 (train monitor) done, [3] pass 1 done.
__device__ long long g_loss_ts[4];

// ---------------------------------------------------------------- period forward -------
// One workgroup (PER_NT threads) per (job, period). When the period has at most
// PER_NT * PER_RB compact rows (the usual case), all of its rows are loaded into registers
// before any use -- one memory round trip instead of one per strided iteration.
#define PER_NT 512
#define PER_RB 8
// store_wn: also write the zero-mean weights w' into the dense [T][N] wn (read only by the host-side
// consumers -- evaluate, the module API, the ensemble export -- never by the epoch's own kernels:
// the epoch graphs skip the scattered stores)
// stage: 0 the whole pass; sharded jobs (LossJob::xs) run it as three launches around the ranks'
// sums (loss.h launch_period_fwd): 1 local sum w, 2 local sums of w' (mu from the global sum),
// 3 P / SDF / portfolio / residual statistics from the global sums.
__global__ __launch_bounds__(PER_NT) void k_period_fwd(const LossJob* __restrict__ jobs, int store_wn, int stage) {
  const LossJob& J = jobs[blockIdx.y];
  const int t = blockIdx.x;
  // the fused forward that produced w has finished (stream order): rearm its progress counter
  if (stage <= 1 && J.prog_reset && t == 0 && threadIdx.x == 0) gp(J.prog_reset)[0] = 0;
  if (t >= J.T) return;
  __shared__ float red[PER_NT / 64];
  const int N = J.N;
  const float invN = gp(J.invNt)[t];
  auto finish = [&](float s_wr, float s_abs, float s_ww) {     // (thread 0)
    const float p = J.weighted ? s_wr * invN * J.Nbar : s_wr;
    gp(J.P)[t] = p;
    gp(J.sdfv)[t] = 1.f + p;
    if (gp(J.port)) gp(J.port)[t] = s_wr / fmaxf(s_abs, 1e-8f);
    if (gp(J.rstat)) {
      gp(J.rstat)[4 * t + 0] = s_ww;
      gp(J.rstat)[4 * t + 1] = s_wr;
    }
  };
  if (stage == 3) {
    if (threadIdx.x == 0) {
      const auto xs = gp(J.xs);
      finish(xs[J.T + t], xs[2 * J.T + t], xs[3 * J.T + t]);
    }
    return;
  }
  const int r0 = gp(J.row_ptr)[t], r1 = gp(J.row_ptr)[t + 1];   // this period's compact rows
  DLAP_ASSERT(0 <= r0 && r0 <= r1 && r1 <= J.R);
  const auto w = gp(J.w);
  const auto Rc = gp(J.Rc);
  const auto rowti = gp(J.rowti);
  float* wn = gp(J.wn) + (size_t)t * N;
  float s_wr = 0.f, s_abs = 0.f, s_ww = 0.f, mu = 0.f;
  // mu from the period's weight sum: the local rows' (stage 0), published for the ranks' sum
  // (stage 1: nothing else to do), or the ranks' sum (stage 2)
  auto mean_of = [&](float sw) -> bool {
    if (stage == 2) { mu = J.normalize ? gp(J.xs)[t] * invN : 0.f; return true; }
    const float tot = J.normalize ? block_sum<PER_NT>(sw, red) : 0.f;
    if (stage == 1) {
      if (threadIdx.x == 0) gp(J.xs)[t] = tot;
      return false;
    }
    mu = tot * invN;
    return true;
  };
  // A period without valid stocks has no compact rows: r0 == r1, possibly == R (the last
  // period of the split), so the clamped `rr = r0` below would read one element past the end of
  // w / Rc / rowti (and then index wn with a garbage stock). Its sums are all zero.
  if (r1 == r0) {
    // (block-uniform: every thread takes this branch; no barrier is skipped by some threads)
    if (!mean_of(0.f)) return;
  } else if (r1 - r0 <= PER_NT * PER_RB) {
    float wv[PER_RB], rv[PER_RB];
    int iv[PER_RB];
#pragma unroll
    for (int k = 0; k < PER_RB; ++k) {
      const int r = r0 + threadIdx.x + PER_NT * k;
      const int rr = r < r1 ? r : r0;
      wv[k] = w[rr]; rv[k] = Rc[rr]; iv[k] = rowti[rr].y;
    }
    float sw = 0.f;
#pragma unroll
    for (int k = 0; k < PER_RB; ++k) sw += (r0 + (int)threadIdx.x + PER_NT * k < r1) ? wv[k] : 0.f;
    if (!mean_of(sw)) return;
#pragma unroll
    for (int k = 0; k < PER_RB; ++k) {
      if (r0 + (int)threadIdx.x + PER_NT * k >= r1) continue;
      const float v = wv[k] - mu;
      if (store_wn) wn[iv[k]] = v;
      s_wr += v * rv[k];
      s_abs += fabsf(v);
      s_ww += v * v;
    }
  } else {          // very wide period: two passes in chunks of PER_NT * PER_RB rows, each
                    // chunk's loads issued before use (the chunk is L2-hot for the second pass)
    constexpr int CH = PER_NT * PER_RB;
    float sw = 0.f;
    if (J.normalize && stage != 2) {
      for (int c0 = r0; c0 < r1; c0 += CH) {
        float wv[PER_RB];
#pragma unroll
        for (int k = 0; k < PER_RB; ++k) {
          const int r = c0 + threadIdx.x + PER_NT * k;
          wv[k] = w[r < r1 ? r : r0];
        }
#pragma unroll
        for (int k = 0; k < PER_RB; ++k) sw += (c0 + (int)threadIdx.x + PER_NT * k < r1) ? wv[k] : 0.f;
      }
    }
    if (!mean_of(sw)) return;
    for (int c0 = r0; c0 < r1; c0 += CH) {
      float wv[PER_RB], rv[PER_RB];
      int iv[PER_RB];
#pragma unroll
      for (int k = 0; k < PER_RB; ++k) {
        const int r = c0 + threadIdx.x + PER_NT * k;
        const int rr = r < r1 ? r : r0;
        wv[k] = w[rr]; rv[k] = Rc[rr]; iv[k] = rowti[rr].y;
      }
#pragma unroll
      for (int k = 0; k < PER_RB; ++k) {
        if (c0 + (int)threadIdx.x + PER_NT * k >= r1) continue;
        const float v = wv[k] - mu;
        if (store_wn) wn[iv[k]] = v;
        s_wr += v * rv[k];
        s_abs += fabsf(v);
        s_ww += v * v;
      }
    }
  }
  if (threadIdx.x == 0) gp(J.mu)[t] = mu;
  s_wr = block_sum<PER_NT>(s_wr, red);
  s_abs = block_sum<PER_NT>(s_abs, red);
  if (gp(J.rstat) || stage == 2) s_ww = block_sum<PER_NT>(s_ww, red);
  if (threadIdx.x == 0) {
    if (stage == 2) {
      const auto xs = gp(J.xs);
      xs[J.T + t] = s_wr;
      xs[2 * J.T + t] = s_abs;
      xs[3 * J.T + t] = s_ww;
    } else {
      finish(s_wr, s_abs, s_ww);
    }
  }
}

// Sharded jobs: the local loss sums of the dense asset passes -> xs[4T], xs[4T + 1] (summed over
// the ranks by the engine's hook before k_job_metrics reads them).
__global__ __launch_bounds__(256) void k_xs_loss_sums(const LossJob* __restrict__ jobs) {
  const LossJob& J = jobs[blockIdx.x];
  __shared__ float red[4];
  float a, b;
  local_loss_sums<256>(J, a, b, red);
  if (threadIdx.x == 0) {
    gp(J.xs)[4 * J.T] = a;
    gp(J.xs)[4 * J.T + 1] = b;
  }
}

// ---------------------------------------------------------------- asset pass ------------
// Pass 1, grid (ceil(N/64), TCH, jobs): block = 64 stocks x one time chunk; the 4 waves split
// the chunk, reduce in LDS (fixed order) and write partial sums for the chunk:
//   pe[ch][i][k] = sum_{t in chunk} h[t,i,k] R[t,i] SDF_t,  pu[ch][i] = sum R SDF_t.
__global__ __launch_bounds__(256) void k_asset_part(const LossJob* __restrict__ jobs) {
  const LossJob& J = jobs[blockIdx.z];
  const int nblk = (J.N + 63) >> 6;
  if ((int)blockIdx.x >= nblk) return;
  __shared__ float red[4][64][9];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int T = J.T, N = J.N, K = J.K;
  const int ch = blockIdx.y;
  const int ca = (T * ch) / DLAP_TCH, cb = (T * (ch + 1)) / DLAP_TCH;
  const int t0 = ca + ((cb - ca) * wave) / 4, t1 = ca + ((cb - ca) * (wave + 1)) / 4;
  const int i = blockIdx.x * 64 + lane;
  const bool ok = i < N;
  float eu = 0.f;
  float e[8];
  const int kmax = J.h ? K : 0;
  for (int k0 = 0; k0 < max(kmax, 1); k0 += 8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = 0.f;
    const int kn = J.h ? min(8, K - k0) : 0;
    if (ok) {
      if (kn == 8 && (K & 3) == 0) {
        // blocks of AW time steps: every operand of the block is requested before use
        constexpr int AW = 8;
        for (int tb = t0; tb < t1; tb += AW) {
          float rm[AW], sv[AW];
          f32x4 ha[AW], hb[AW];
#pragma unroll
          for (int u = 0; u < AW; ++u) {
            const int t = min(tb + u, t1 - 1);
            const size_t d = (size_t)t * N + i;
            rm[u] = gp(J.Rm)[d];
            sv[u] = gp(J.sdfv)[t];
            const auto hp = gp(J.h) + d * K + k0;
            ha[u] = ld4(hp);
            hb[u] = ld4(hp + 4);
          }
#pragma unroll
          for (int u = 0; u < AW; ++u) {
            const float q = tb + u < t1 ? rm[u] * sv[u] : 0.f;
            if (k0 == 0) eu += q;
#pragma unroll
            for (int k = 0; k < 4; ++k) { e[k] += ha[u][k] * q; e[4 + k] += hb[u][k] * q; }
          }
        }
      } else {
#pragma unroll 4
        for (int t = t0; t < t1; ++t) {
          const size_t d = (size_t)t * N + i;
          const float q = gp(J.Rm)[d] * gp(J.sdfv)[t];
          if (k0 == 0) eu += q;
          for (int k = 0; k < kn; ++k) e[k] += gp(J.h)[d * K + k0 + k] * q;
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) red[wave][lane][k] = e[k];
    red[wave][lane][8] = eu;
    __syncthreads();
    if (wave == 0 && ok) {
      float* pe = gp(J.pe) + ((size_t)ch * N + i) * K;
      for (int k = 0; k < kn; ++k)
        pe[k0 + k] = red[0][lane][k] + red[1][lane][k] + red[2][lane][k] + red[3][lane][k];
      if (k0 == 0) gp(J.pu)[(size_t)ch * N + i] = red[0][lane][8] + red[1][lane][8] + red[2][lane][8] + red[3][lane][8];
    }
  }
}

// Pass 2, grid (ceil(N (K+1) / 256), jobs): one thread per output (stock i, moment k), the
// last "moment" k = K being the unconditional E_unc; the DLAP_TCH chunk partials of an output are
// all requested before they are summed (in chunk order), so the pass is one memory round trip.
// Writes E, E_unc, dL/dE and the block's loss partial sums. Without moments (h == nullptr: the
// unconditional training loss) only the E_unc outputs exist.
__global__ __launch_bounds__(256) void k_asset_red(const LossJob* __restrict__ jobs) {
  const LossJob& J = jobs[blockIdx.y];
  const int N = J.N, K = J.K, kk = J.h ? K + 1 : 1;
  if ((int)blockIdx.x >= asset_red_blocks(J)) return;          // block-uniform
  __shared__ float red[4];
  const int o = blockIdx.x * 256 + threadIdx.x;
  const bool ok = o < N * kk;
  const int i = ok ? o / kk : 0, k = ok ? o - i * kk : 0;
  const bool unc = k == kk - 1;
  float lc = 0.f, lu = 0.f;
  if (ok) {
    float p[DLAP_TCH];
#pragma unroll
    for (int ch = 0; ch < DLAP_TCH; ++ch)
      p[ch] = unc ? gp(J.pu)[(size_t)ch * N + i] : gp(J.pe)[((size_t)ch * N + i) * K + k];
    float v = 0.f;
#pragma unroll
    for (int ch = 0; ch < DLAP_TCH; ++ch) v += p[ch];
    v *= gp(J.invT)[i];
    if (unc) {
      gp(J.Eu)[i] = v;
      if (gp(J.dEu)) gp(J.dEu)[i] = J.coef_u * v;
      lu = v * v;
    } else {
      gp(J.E)[(size_t)i * K + k] = v;
      if (gp(J.dE)) gp(J.dE)[(size_t)i * K + k] = J.coef_c * v;
      lc = v * v;
    }
  }
  lc = block_sum<256>(lc, red);
  lu = block_sum<256>(lu, red);
  if (threadIdx.x == 0) {
    gp(J.part)[2 * blockIdx.x + 0] = lc;
    gp(J.part)[2 * blockIdx.x + 1] = lu;
  }
}

// One-pass asset reduction, grid (ceil(N / AF_S), jobs), 256 threads = AF_S stocks x 16 time
// lanes: each thread sums E over its time lane's periods (blocks of AF_U periods, every operand
// requested before use), the 16 lanes are summed in LDS in a fixed order, and the first lane of
// each stock writes E, E_unc, dL/dE and the block's loss partials -- the whole time axis of a
// stock stays in one workgroup, so no second reduction launch (k_asset_red) is needed.
#define AF_U 4
__global__ __launch_bounds__(256) void k_asset_full(const LossJob* __restrict__ jobs) {
  const LossJob& J = jobs[blockIdx.y];
  const int N = J.N, K = J.K, T = J.T;
  if ((int)blockIdx.x * AF_S >= N) return;                      // block-uniform
  __shared__ float red[16][AF_S][9];
  __shared__ float lred[4];
  const int s = threadIdx.x % AF_S, tl = threadIdx.x / AF_S;
  const int i = blockIdx.x * AF_S + s;
  const bool ok = i < N;
  const int ic = ok ? i : N - 1;
  const int kmax = J.h ? K : 0;
  const float invT = gp(J.invT)[ic];
  float lc = 0.f, lu = 0.f;
  for (int k0 = 0; k0 < max(kmax, 1); k0 += 8) {
    const int kn = J.h ? min(8, K - k0) : 0;
    float e[8], eu = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = 0.f;
    if (kn == 8 && (K & 3) == 0) {
      for (int tb = tl; tb < T; tb += 16 * AF_U) {
        float q[AF_U];
        f32x4 ha[AF_U], hb[AF_U];
#pragma unroll
        for (int u = 0; u < AF_U; ++u) {
          const int t = tb + 16 * u;
          const int tc = t < T ? t : T - 1;
          const size_t d = (size_t)tc * N + ic;
          q[u] = t < T ? gp(J.Rm)[d] * gp(J.sdfv)[tc] : 0.f;
          const auto hp = gp(J.h) + d * K + k0;
          ha[u] = ld4(hp);
          hb[u] = ld4(hp + 4);
        }
#pragma unroll
        for (int u = 0; u < AF_U; ++u) {
          eu += q[u];
#pragma unroll
          for (int k = 0; k < 4; ++k) { e[k] += ha[u][k] * q[u]; e[4 + k] += hb[u][k] * q[u]; }
        }
      }
    } else {
      for (int tb = tl; tb < T; tb += 16 * AF_U) {
        float q[AF_U];
#pragma unroll
        for (int u = 0; u < AF_U; ++u) {
          const int t = tb + 16 * u;
          const int tc = t < T ? t : T - 1;
          q[u] = t < T ? gp(J.Rm)[(size_t)tc * N + ic] * gp(J.sdfv)[tc] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < AF_U; ++u) {
          const int t = tb + 16 * u;
          eu += q[u];
          if (t < T)
            for (int k = 0; k < kn; ++k) e[k] += gp(J.h)[((size_t)t * N + ic) * K + k0 + k] * q[u];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) red[tl][s][k] = e[k];
    red[tl][s][8] = eu;
    __syncthreads();
    if (tl == 0 && ok) {
      for (int k = 0; k < kn; ++k) {
        float v = 0.f;
#pragma unroll
        for (int l = 0; l < 16; ++l) v += red[l][s][k];
        v *= invT;
        gp(J.E)[(size_t)i * K + k0 + k] = v;
        if (gp(J.dE)) gp(J.dE)[(size_t)i * K + k0 + k] = J.coef_c * v;
        lc += v * v;
      }
      if (k0 == 0) {
        float v = 0.f;
#pragma unroll
        for (int l = 0; l < 16; ++l) v += red[l][s][8];
        v *= invT;
        gp(J.Eu)[i] = v;
        if (gp(J.dEu)) gp(J.dEu)[i] = J.coef_u * v;
        lu = v * v;
      }
    }
  }
  lc = block_sum<256>(lc, lred);
  lu = block_sum<256>(lu, lred);
  if (threadIdx.x == 0) {
    gp(J.part)[2 * blockIdx.x + 0] = lc;
    gp(J.part)[2 * blockIdx.x + 1] = lu;
  }
}

// ---------------------------------------------------------------- period backward ------
// Gram mode: (Gc s)_t and (Gu s)_t for period t in fp64, their loss terms s_t (G s)_t into
// gpart, and dL/dSDF_t of the job's training loss (phase 1: L_unc, 3: L_cond; 0: none).
DLAP_DEV float gram_period(const LossJob& J, int t, double* redd) {
  const int T = J.T;
  const size_t T2 = (size_t)T * T;
  const auto G = gp(J.G) + (size_t)t * T;
  const auto sv = gp(J.sdfv);
  const bool cond = J.h != nullptr;
  double vc = 0.0, vu = 0.0;
  for (int u = threadIdx.x; u < T; u += PER_NT) {
    const double s = (double)sv[u];
    if (cond) vc += G[u] * s;
    vu += G[T2 + u] * s;
  }
  if (cond) vc = block_sum_d<PER_NT>(vc, redd);
  vu = block_sum_d<PER_NT>(vu, redd);
  if (threadIdx.x == 0) {
    const double st = (double)sv[t];
    gp(J.gpart)[2 * t + 0] = cond ? st * vc : 0.0;
    gp(J.gpart)[2 * t + 1] = st * vu;
  }
  // coef_c = +-2/(KN), coef_u = 2/N (see Engine::loss_job); dL/dSDF = coef (G s)
  if (J.phase == 1) return (float)((double)J.coef_u * vu);
  if (J.phase == 2 || J.phase == 3) return (float)((double)J.coef_c * vc);
  return 0.f;
}

// METRICS: one extra workgroup (the last, blockIdx.x == gridDim.x - 1) computes the job's
// scalar metrics (k_job_metrics) beside the period workgroups: one launch less on the
// training chain.
template <bool METRICS>
__global__ __launch_bounds__(PER_NT) void k_period_bwd(const LossJob* __restrict__ jobs) {
  const LossJob& J = jobs[blockIdx.y];
  const int t = blockIdx.x;
  __shared__ float red[PER_NT / 64];
  if constexpr (METRICS) {
    __shared__ float ret[DLAP_MAX_T];
    if (t == (int)gridDim.x - 1) { job_metrics_body<PER_NT>(J, red, ret, g_loss_ts); return; }
  }
  if (t >= J.T) return;
  const int N = J.N, K = J.K;
  const size_t base = (size_t)t * N;
  const int r0 = gp(J.row_ptr)[t], r1 = gp(J.row_ptr)[t + 1];
  DLAP_ASSERT(0 <= r0 && r0 <= r1 && r1 <= J.R);
  float sg = 0.f;                  // Gram mode: dL/dSDF_t
  if (J.gram) {
    __shared__ double redd[PER_NT / 64];
    sg = gram_period(J, t, redd);
    if (J.phase == 0) return;      // evaluation: loss terms only
  }
  // no compact rows in this period (all stocks masked): no dL/dw to write, and the clamped
  // row index of the loads below would point past the end of the arrays when r0 == R
  if (r1 == r0) return;            // block-uniform, before any barrier
  const auto rowti = gp(J.rowti);
  const auto Rc = gp(J.Rc);
  const auto invT = gp(J.invT);
  // per-row dL/dS contribution: g_i R_i / T_i with g = dE_u (phase 1) or sum_k dE[i,k] h[t,i,k]
  auto row_g = [&](int i) -> float {
    if (J.phase == 1) return gp(J.dEu)[i];
    const auto hp = gp(J.h) + (base + i) * K;
    const auto de = gp(J.dE) + (size_t)i * K;
    float g = 0.f;
    for (int k = 0; k < K; ++k) g += de[k] * hp[k];
    return g;
  };
  constexpr int RB = 4;
  const bool fast = r1 - r0 <= PER_NT * RB;
  // one chunk of PER_NT * RB rows: every row's operands are requested before any is used
  // (2 dependent round trips per chunk); periods wider than one chunk loop over chunks
  auto chunk_sum = [&](int c0, float (&rv)[RB]) -> float {
    int iv[RB];
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const int r = c0 + threadIdx.x + PER_NT * k;
      const int rr = r < r1 ? r : r0;
      iv[k] = rowti[rr].y;
      rv[k] = Rc[rr];
    }
    float gv[RB], tv[RB];
    if (J.phase != 1 && K == 8) {
      f32x4 d0[RB], d1[RB], h0[RB], h1[RB];
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const auto hp = gp(J.h) + (base + iv[k]) * 8;
        const auto de = gp(J.dE) + (size_t)iv[k] * 8;
        d0[k] = ld4(de); d1[k] = ld4(de + 4); h0[k] = ld4(hp); h1[k] = ld4(hp + 4);
        tv[k] = invT[iv[k]];
      }
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        float g = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) g += d0[k][e] * h0[k][e] + d1[k][e] * h1[k][e];
        gv[k] = g;
      }
    } else {
#pragma unroll
      for (int k = 0; k < RB; ++k) { gv[k] = row_g(iv[k]); tv[k] = invT[iv[k]]; }
    }
    float part = 0.f;
#pragma unroll
    for (int k = 0; k < RB; ++k)
      if (c0 + (int)threadIdx.x + PER_NT * k < r1) part += gv[k] * rv[k] * tv[k];
    return part;
  };
  float rv[RB];
  float s = 0.f;
  if (J.gram) {
    s = sg;
    if (fast) {
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const int r = r0 + threadIdx.x + PER_NT * k;
        rv[k] = Rc[r < r1 ? r : r0];
      }
    }
  } else {
    if (fast) {
      s = chunk_sum(r0, rv);
    } else {
      for (int c0 = r0; c0 < r1; c0 += PER_NT * RB) {
        float rt[RB];
        s += chunk_sum(c0, rt);
      }
    }
    s = block_sum<PER_NT>(s, red);
  }
  const float c = J.weighted ? s * J.Nbar * gp(J.invNt)[t] : s;   // dL/dS_t with S_t = sum w' R m
  // optional residual-loss gradient wrt w' (valid stocks of period t)
  float rcoef = 0.f, beta = 0.f;
  if (J.res_factor > 0.f) {
    float lres, inv_b, n1;
    residual_stats(J, lres, inv_b, n1);
    const float n = gp(J.Nt)[t], ww = gp(J.rstat)[4 * t + 0], rw = gp(J.rstat)[4 * t + 1];
    if (n >= 2.f && ww > 1e-8f && n1 > 0.f) {
      beta = rw / ww;
      rcoef = J.res_factor * inv_b / n1 * (-2.f / n) * beta;   // d/dw'_i = rcoef * (R_i - beta w'_i)
    }
  }
  const float mu = gp(J.mu)[t];
  float gres_mean = 0.f;
  if (rcoef != 0.f && J.normalize && J.xs) {
    // sharded: the period's sum over every rank's stocks, sum (R_i - beta w'_i) = N_t mean R
    // (the zero-mean weights sum to 0)
    gres_mean = rcoef * gp(J.meanR)[t];
  } else if (rcoef != 0.f && J.normalize) {
    float sg = 0.f;
    for (int rr = r0 + threadIdx.x; rr < r1; rr += PER_NT) sg += Rc[rr] - beta * (gp(J.w)[rr] - mu);
    sg = block_sum<PER_NT>(sg, red);
    gres_mean = rcoef * sg * gp(J.invNt)[t];
  }
  const float mR = J.normalize ? gp(J.meanR)[t] : 0.f;
  if (fast && rcoef == 0.f) {
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const int r = r0 + threadIdx.x + PER_NT * k;
      if (r < r1) gp(J.dw)[r] = c * (rv[k] - mR);
    }
  } else if (rcoef == 0.f) {
    for (int c0 = r0; c0 < r1; c0 += PER_NT * RB) {
      float rt[RB];
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const int r = c0 + threadIdx.x + PER_NT * k;
        rt[k] = Rc[r < r1 ? r : r0];
      }
#pragma unroll
      for (int k = 0; k < RB; ++k) {
        const int r = c0 + threadIdx.x + PER_NT * k;
        if (r < r1) gp(J.dw)[r] = c * (rt[k] - mR);
      }
    }
  } else {
    for (int rr = r0 + threadIdx.x; rr < r1; rr += PER_NT) {
      const float R = Rc[rr];
      float g = c * (R - mR);
      if (rcoef != 0.f) g += rcoef * (R - beta * (gp(J.w)[rr] - mu)) - gres_mean;
      gp(J.dw)[rr] = g;
    }
  }
}

__global__ __launch_bounds__(256) void k_job_metrics(const LossJob* __restrict__ jobs) {
  __shared__ float red[4];
  __shared__ float ret[DLAP_MAX_T];
  job_metrics_body<256>(jobs[blockIdx.x], red, ret, g_loss_ts);
}

std::vector<long long> loss_timestamps() {
  std::vector<long long> v(4);
  HIP_OK(hipMemcpyFromSymbol(v.data(), HIP_SYMBOL(g_loss_ts), sizeof(long long) * 4));
  return v;
}

// ---------------------------------------------------------------- launchers ------------
void launch_period_fwd(const LossJob* jobs, int njobs, int tmax, hipStream_t st, bool store_wn, int stage) {
  hipLaunchKernelGGL(k_period_fwd, dim3(tmax, njobs), dim3(PER_NT), 0, st, jobs, (int)store_wn, stage);
  HIP_OK(hipGetLastError());
}
void launch_xs_loss_sums(const LossJob* jobs, int njobs, hipStream_t st) {
  hipLaunchKernelGGL(k_xs_loss_sums, dim3(njobs), dim3(256), 0, st, jobs);
  HIP_OK(hipGetLastError());
}
bool asset_full_default() {
  static const bool on = [] { const char* v = std::getenv("DLAP_ASSET_FULL"); return !(v && *v == '0'); }();
  return on;
}
void launch_asset(const LossJob* jobs, int njobs, int nmax, int kmax, hipStream_t st, bool full) {
  if (full) {                     // (the job tables were built with asset_full = 1)
    hipLaunchKernelGGL(k_asset_full, dim3((nmax + AF_S - 1) / AF_S, njobs), dim3(256), 0, st, jobs);
    HIP_OK(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL(k_asset_part, dim3((nmax + 63) / 64, DLAP_TCH, njobs), dim3(256), 0, st, jobs);
  HIP_OK(hipGetLastError());
  hipLaunchKernelGGL(k_asset_red, dim3((nmax * (kmax + 1) + 255) / 256, njobs), dim3(256), 0, st, jobs);
  HIP_OK(hipGetLastError());
}
void launch_period_bwd(const LossJob* jobs, int njobs, int tmax, hipStream_t st, bool metrics) {
  if (metrics) hipLaunchKernelGGL(k_period_bwd<true>, dim3(tmax + 1, njobs), dim3(PER_NT), 0, st, jobs);
  else hipLaunchKernelGGL(k_period_bwd<false>, dim3(tmax, njobs), dim3(PER_NT), 0, st, jobs);
  HIP_OK(hipGetLastError());
}
void launch_job_metrics(const LossJob* jobs, int njobs, hipStream_t st) {
  hipLaunchKernelGGL(k_job_metrics, dim3(njobs), dim3(256), 0, st, jobs);
  HIP_OK(hipGetLastError());
}

// ---------------------------------------------------------------- ensemble (K11) --------
// Post-all-gather ensemble portfolio of `/root/reference/src/evaluate_ensemble.py:137-166` on the
// device: one workgroup per period t over G models' L1-normalised weights W [G][T][N]:
//   a_i = mean_g W[g,t,i];  s = sum_i |a_i| m_i (fp64);  q_i = s > 1e-8 ? a_i / s : a_i;
//   port[t] = sum_i q_i R_i m_i,  port_ind[g][t] = sum_i W[g,t,i] R_i m_i   (fp64 sums)
// The (tiny) Sharpe ratios of these [T] series are taken on the host.

__global__ __launch_bounds__(256) void k_ensemble(const float* __restrict__ W, int G, int T, int N,
                                                  const float* __restrict__ R, const float* __restrict__ mask,
                                                  float* __restrict__ port, float* __restrict__ port_ind) {
  __shared__ double red[4];
  const int t = blockIdx.x;
  if (t >= T) return;
  const size_t tn = (size_t)t * N;
  const float invG = 1.f / (float)G;
  double sa = 0.0;
  for (int i = threadIdx.x; i < N; i += 256) {
    float a = 0.f;
    for (int g = 0; g < G; ++g) a += gp(W)[(size_t)g * T * N + tn + i];
    a *= invG;
    sa += fabs((double)a) * (double)gp(mask)[tn + i];
  }
  const double s = block_sum_d<256>(sa, red);
  double pr = 0.0;
  for (int i = threadIdx.x; i < N; i += 256) {
    float a = 0.f;
    for (int g = 0; g < G; ++g) a += gp(W)[(size_t)g * T * N + tn + i];
    a *= invG;
    const float q = s > 1e-8 ? (float)((double)a / s) : a;
    pr += (double)q * (double)gp(R)[tn + i] * (double)gp(mask)[tn + i];
  }
  pr = block_sum_d<256>(pr, red);
  if (threadIdx.x == 0) gp(port)[t] = (float)pr;
  for (int g = 0; g < G; ++g) {
    double pg = 0.0;
    for (int i = threadIdx.x; i < N; i += 256)
      pg += (double)gp(W)[(size_t)g * T * N + tn + i] * (double)gp(R)[tn + i] * (double)gp(mask)[tn + i];
    pg = block_sum_d<256>(pg, red);
    if (threadIdx.x == 0) gp(port_ind)[(size_t)g * T + t] = (float)pg;
  }
}

void launch_ensemble(const float* W, int G, int T, int N, const float* R, const float* mask, float* port,
                     float* port_ind, hipStream_t st) {
  if (T <= 0 || G <= 0) return;
  hipLaunchKernelGGL(k_ensemble, dim3(T), dim3(256), 0, st, W, G, T, N, R, mask, port, port_ind);
  HIP_OK(hipGetLastError());
}
