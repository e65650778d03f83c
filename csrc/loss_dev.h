// Device-side loss helpers shared by the loss kernels (k_loss.hip) and the fused backward tail
// (k_rnn.hip, which computes the train split's job metrics in one of its blocks).
#pragma once
#include "common.h"
#include "loss.h"

// ---------------------------------------------------------------- residual loss --------
// L_res = mean_{t in S1} resid_t / max(mean_{t in S2} Rsq_t, 1e-8)
//   S2 = {n_t >= 2},  S1 = S2 and ww_t > 1e-8,  resid_t = (RR - Rw^2/ww)/n_t,  Rsq_t = RR/n_t.
DLAP_DEV void residual_stats(const LossJob& J, float& lres, float& inv_b, float& n1) {
  float a = 0.f, b = 0.f, c1 = 0.f, c2 = 0.f;
  for (int t = 0; t < J.T; ++t) {
    const float n = gp(J.Nt)[t];
    if (n < 2.f) continue;
    const float ww = gp(J.rstat)[4 * t + 0], rw = gp(J.rstat)[4 * t + 1], rr = gp(J.RR)[t];
    b += rr / n; c2 += 1.f;
    if (ww > 1e-8f) { a += (rr - rw * rw / ww) / n; c1 += 1.f; }
  }
  if (c1 == 0.f) { lres = 0.f; inv_b = 0.f; n1 = 0.f; return; }
  const float B = fmaxf(b / c2, 1e-8f);
  lres = (a / c1) / B;
  inv_b = 1.f / B;
  n1 = c1;
}

// number of loss partials the asset pass leaves in J.part (read by final_losses)
#define AF_S 16            // k_asset_full: stocks per workgroup (x 16 time lanes)
DLAP_DEV int asset_red_blocks(const LossJob& J) {
  return J.asset_full ? (J.N + AF_S - 1) / AF_S : (J.N * (J.h ? J.K + 1 : 1) + 255) >> 8;
}

template <int NT>
DLAP_DEV double block_sum_d(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += red[i];
  return s;
}

// Block-wide (256 threads) fixed-order sum of the asset blocks' loss partials: every thread
// takes a strided share (all loads in flight at once, instead of 2 * nblk dependent round trips
// on one thread), then the fixed-order block reduction.
template <int NT>
DLAP_DEV double block_sum_d(double v, double* red);

// (the local loss sums of the dense asset passes, before the division by K N / N)
template <int NT>
DLAP_DEV void local_loss_sums(const LossJob& J, float& a, float& b, float* red) {
  const int nblk = asset_red_blocks(J);
  a = 0.f; b = 0.f;
  for (int k = threadIdx.x; k < nblk; k += NT) { a += gp(J.part)[2 * k]; b += gp(J.part)[2 * k + 1]; }
  a = block_sum<NT>(a, red);
  b = block_sum<NT>(b, red);
}

template <int NT>
DLAP_DEV void final_losses(const LossJob& J, float& lc, float& lu, float* red) {
  if (J.gram) {        // fixed-order fp64 sum of the per-period quadratic-form terms
    __shared__ double redd[NT / 64];
    double a = 0.0, b = 0.0;
    for (int t = threadIdx.x; t < J.T; t += NT) { a += gp(J.gpart)[2 * t]; b += gp(J.gpart)[2 * t + 1]; }
    a = block_sum_d<NT>(a, redd);
    b = block_sum_d<NT>(b, redd);
    lc = J.h ? (float)(a / ((double)J.K * (double)J.Nnorm)) : 0.f;
    lu = (float)(b / (double)J.Nnorm);
    return;
  }
  float a, b;
  if (J.xs) {          // sharded: the loss sums of every rank's stocks (launch_xs_loss_sums + hook)
    a = gp(J.xs)[4 * J.T];
    b = gp(J.xs)[4 * J.T + 1];
  } else {
    local_loss_sums<NT>(J, a, b, red);
  }
  lc = J.h ? a / ((float)J.K * J.Nnorm) : 0.f;
  lu = b / J.Nnorm;
}

// ts: in-kernel timestamps (k_job_metrics' g_loss_ts), or nullptr
#define MET_TS(slot) do { if (ts && threadIdx.x == 0 && blockIdx.x == gridDim.x - 1) ts[slot] = wall_clock64(); } while (0)

// ---------------------------------------------------------------- per-job scalars -------
// scal layout: see loss.h (SC_*).
template <int NT>
DLAP_DEV void job_metrics_body(const LossJob& J, float* red, float* ret, long long* ts = nullptr) {
  const int T = J.T;
  MET_TS(0);
  float lc, lu;
  final_losses<NT>(J, lc, lu, red);
  MET_TS(1);
  if (threadIdx.x == 0) {
    float lres = 0.f, inv_b, n1;
    if (J.res_factor > 0.f) residual_stats(J, lres, inv_b, n1);
    st_wt(gp(J.scal) + SC_LCOND, lc);
    st_wt(gp(J.scal) + SC_LUNC, lu);
    st_wt(gp(J.scal) + SC_LRES, lres);
  }
  // Sharpe of the weighted training portfolio P (train monitor) and of the L1 portfolio.
  for (int pass = 0; pass < 2; ++pass) {
    const float* src = pass == 0 ? gp(J.P) : gp(J.port);
    if (!src) continue;
    for (int t = threadIdx.x; t < T; t += NT) ret[t] = src[t];
    __syncthreads();
    float s = 0.f;
    for (int t = threadIdx.x; t < T; t += NT) s += ret[t];
    s = block_sum<NT>(s, red);
    const float mean = s / (float)T;
    float v = 0.f;
    for (int t = threadIdx.x; t < T; t += NT) { const float x = ret[t] - mean; v += x * x; }
    v = block_sum<NT>(v, red);
    if (threadIdx.x == 0) {
      const float sd_u = T > 1 ? sqrtf(v / (float)(T - 1)) : __builtin_nanf("");
      const float sharpe = (sd_u < 1e-8f) ? 0.f : mean / sd_u;
      if (pass == 0) {
        st_wt(gp(J.scal) + SC_TRAIN_SHARPE, sharpe);
      } else {
        st_wt(gp(J.scal) + SC_SHARPE, sharpe);
        st_wt(gp(J.scal) + SC_MEAN, mean);
        st_wt(gp(J.scal) + SC_STD, sqrtf(v / (float)T));
      }
    }
    if (pass == 1 && threadIdx.x < 64) {
      // max drawdown of cumprod(1 + r) on wave 0: each lane owns a contiguous run of periods;
      // prefix product and prefix running-max across lanes by shuffle scans (replaces a
      // T-step serial loop on one thread; products associate differently: fp32 rounding only)
      const int lane = threadIdx.x, per = (T + 63) >> 6;
      const int t0 = min(T, lane * per), t1 = min(T, t0 + per);
      float prod = 1.f;
      for (int t = t0; t < t1; ++t) prod *= 1.f + ret[t];
      float incl = prod;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float u = __shfl_up(incl, o, 64);
        if (lane >= o) incl *= u;
      }
      float base = __shfl_up(incl, 1, 64);
      if (lane == 0) base = 1.f;
      float cum = base, lmax = -INFINITY;
      for (int t = t0; t < t1; ++t) { cum *= 1.f + ret[t]; lmax = fmaxf(lmax, cum); }
      float pmax = lmax;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float u = __shfl_up(pmax, o, 64);
        if (lane >= o) pmax = fmaxf(pmax, u);
      }
      float peak = __shfl_up(pmax, 1, 64);
      if (lane == 0) peak = -INFINITY;
      cum = base;
      float mdd = 0.f;
      for (int t = t0; t < t1; ++t) {
        cum *= 1.f + ret[t];
        peak = t == 0 ? cum : fmaxf(peak, cum);
        mdd = fminf(mdd, (cum - peak) / peak);
      }
      mdd = wave_min(mdd);
      if (lane == 0) st_wt(gp(J.scal) + SC_MDD, mdd);
    }
    __syncthreads();
    MET_TS(2 + pass);
  }
}

