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
//   k_period_bwd  one workgroup per (job, period): dL/dSDF_t and the analytic gradient of
//                 the zero-mean normalisation, dL/dw_raw = m c_t (R - mean_t R) (+ residual)
//   k_job_metrics one workgroup per job: scalar losses, Sharpe (unbiased std, 1e-8 guard),
//                 max drawdown (cumprod scan), mean/std of the evaluation returns
#include "common.h"
#include "loss.h"

// ---------------------------------------------------------------- period forward -------
__global__ __launch_bounds__(256) void k_period_fwd(const LossJob* __restrict__ jobs) {
  const LossJob& J = jobs[blockIdx.y];
  const int t = blockIdx.x;
  if (t >= J.T) return;
  __shared__ float red[4];
  const int N = J.N;
  const int r0 = gp(J.row_ptr)[t], r1 = gp(J.row_ptr)[t + 1];   // this period's compact rows
  float sw = 0.f;
  if (J.normalize) {
    for (int r = r0 + threadIdx.x; r < r1; r += 256) sw += gp(J.w)[r];
    sw = block_sum<256>(sw, red);
  }
  const float mu = J.normalize ? sw * gp(J.invNt)[t] : 0.f;
  float s_wr = 0.f, s_abs = 0.f, s_ww = 0.f;
  float* wn = gp(J.wn) + (size_t)t * N;
  for (int r = r0 + threadIdx.x; r < r1; r += 256) {
    const float v = gp(J.w)[r] - mu;
    wn[gp(J.rowti)[r].y] = v;
    s_wr += v * gp(J.Rc)[r];
    s_abs += fabsf(v);
    s_ww += v * v;
  }
  if (threadIdx.x == 0) gp(J.mu)[t] = mu;
  s_wr = block_sum<256>(s_wr, red);
  s_abs = block_sum<256>(s_abs, red);
  if (gp(J.rstat)) s_ww = block_sum<256>(s_ww, red);
  if (threadIdx.x == 0) {
    const float p = J.weighted ? s_wr * gp(J.invNt)[t] * J.Nbar : s_wr;
    gp(J.P)[t] = p;
    gp(J.sdfv)[t] = 1.f + p;
    if (gp(J.port)) gp(J.port)[t] = s_wr / fmaxf(s_abs, 1e-8f);
    if (gp(J.rstat)) {
      gp(J.rstat)[4 * t + 0] = s_ww;
      gp(J.rstat)[4 * t + 1] = s_wr;
    }
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
#pragma unroll 4
      for (int t = t0; t < t1; ++t) {
        const size_t d = (size_t)t * N + i;
        const float q = gp(J.Rm)[d] * gp(J.sdfv)[t];
        if (k0 == 0) eu += q;
        if (kn == 8 && (K & 3) == 0) {
          const float* hp = gp(J.h) + d * K + k0;
          const f32x4 a = *reinterpret_cast<const f32x4*>(hp);
          const f32x4 b = *reinterpret_cast<const f32x4*>(hp + 4);
#pragma unroll
          for (int k = 0; k < 4; ++k) { e[k] += a[k] * q; e[4 + k] += b[k] * q; }
        } else {
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

// Pass 2, grid (ceil(N/256), jobs): thread per stock; sums the chunks in order, writes
// E, E_unc, dL/dE and the block's loss partial sums.
__global__ __launch_bounds__(256) void k_asset_red(const LossJob* __restrict__ jobs) {
  const LossJob& J = jobs[blockIdx.y];
  const int N = J.N, K = J.K;
  if ((int)blockIdx.x * 256 >= N) return;
  __shared__ float red[4];
  const int i = blockIdx.x * 256 + threadIdx.x;
  const bool ok = i < N;
  float lc = 0.f, lu = 0.f;
  if (ok) {
    const float invT = gp(J.invT)[i];
    float u = 0.f;
    for (int ch = 0; ch < DLAP_TCH; ++ch) u += gp(J.pu)[(size_t)ch * N + i];
    u *= invT;
    gp(J.Eu)[i] = u;
    if (gp(J.dEu)) gp(J.dEu)[i] = J.coef_u * u;
    lu = u * u;
    if (gp(J.h)) {
      for (int k = 0; k < K; ++k) {
        float v = 0.f;
        for (int ch = 0; ch < DLAP_TCH; ++ch) v += gp(J.pe)[((size_t)ch * N + i) * K + k];
        v *= invT;
        gp(J.E)[(size_t)i * K + k] = v;
        if (gp(J.dE)) gp(J.dE)[(size_t)i * K + k] = J.coef_c * v;
        lc += v * v;
      }
    }
  }
  lc = block_sum<256>(lc, red);
  lu = block_sum<256>(lu, red);
  if (threadIdx.x == 0) {
    gp(J.part)[2 * blockIdx.x + 0] = lc;
    gp(J.part)[2 * blockIdx.x + 1] = lu;
  }
}

DLAP_DEV void final_losses(const LossJob& J, float& lc, float& lu) {
  const int nblk = (J.N + 255) >> 8;
  float a = 0.f, b = 0.f;
  for (int k = 0; k < nblk; ++k) { a += gp(J.part)[2 * k]; b += gp(J.part)[2 * k + 1]; }
  lc = J.h ? a / ((float)J.K * (float)J.N) : 0.f;
  lu = b / (float)J.N;
}

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

// ---------------------------------------------------------------- period backward ------
__global__ __launch_bounds__(256) void k_period_bwd(const LossJob* __restrict__ jobs) {
  const LossJob& J = jobs[blockIdx.y];
  const int t = blockIdx.x;
  if (t >= J.T) return;
  __shared__ float red[4];
  const int N = J.N, K = J.K;
  const size_t base = (size_t)t * N;
  const int r0 = gp(J.row_ptr)[t], r1 = gp(J.row_ptr)[t + 1];
  float s = 0.f;
  for (int rr = r0 + threadIdx.x; rr < r1; rr += 256) {
    const int i = gp(J.rowti)[rr].y;
    const float r = gp(J.Rc)[rr];
    float g;
    if (J.phase == 1) {
      g = gp(J.dEu)[i];
    } else {
      g = 0.f;
      const float* hp = gp(J.h) + (base + i) * K;
      const float* de = gp(J.dE) + (size_t)i * K;
      for (int k = 0; k < K; ++k) g += de[k] * hp[k];
    }
    s += g * r * gp(J.invT)[i];
  }
  s = block_sum<256>(s, red);
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
  // mean over valid stocks of the residual gradient (for the normalisation Jacobian)
  const float mu = gp(J.mu)[t];
  float gres_mean = 0.f;
  if (rcoef != 0.f && J.normalize) {
    float sg = 0.f;
    for (int rr = r0 + threadIdx.x; rr < r1; rr += 256) sg += gp(J.Rc)[rr] - beta * (gp(J.w)[rr] - mu);
    sg = block_sum<256>(sg, red);
    gres_mean = rcoef * sg * gp(J.invNt)[t];
  }
  const float mR = J.normalize ? gp(J.meanR)[t] : 0.f;
  for (int rr = r0 + threadIdx.x; rr < r1; rr += 256) {
    const float R = gp(J.Rc)[rr];
    float g = c * (R - mR);
    if (rcoef != 0.f) g += rcoef * (R - beta * (gp(J.w)[rr] - mu)) - gres_mean;
    gp(J.dw)[rr] = g;
  }
}

// ---------------------------------------------------------------- per-job scalars -------
// scal layout: see loss.h (SC_*).
__global__ __launch_bounds__(256) void k_job_metrics(const LossJob* __restrict__ jobs) {
  const LossJob& J = jobs[blockIdx.x];
  __shared__ float red[4];
  __shared__ float ret[DLAP_MAX_T];
  const int T = J.T;
  if (threadIdx.x == 0) {
    float lc, lu;
    final_losses(J, lc, lu);
    float lres = 0.f, inv_b, n1;
    if (J.res_factor > 0.f) residual_stats(J, lres, inv_b, n1);
    gp(J.scal)[SC_LCOND] = lc;
    gp(J.scal)[SC_LUNC] = lu;
    gp(J.scal)[SC_LRES] = lres;
  }
  // Sharpe of the weighted training portfolio P (train monitor) and of the L1 portfolio.
  for (int pass = 0; pass < 2; ++pass) {
    const float* src = pass == 0 ? gp(J.P) : gp(J.port);
    if (!src) continue;
    for (int t = threadIdx.x; t < T; t += 256) ret[t] = src[t];
    __syncthreads();
    float s = 0.f;
    for (int t = threadIdx.x; t < T; t += 256) s += ret[t];
    s = block_sum<256>(s, red);
    const float mean = s / (float)T;
    float v = 0.f;
    for (int t = threadIdx.x; t < T; t += 256) { const float x = ret[t] - mean; v += x * x; }
    v = block_sum<256>(v, red);
    if (threadIdx.x == 0) {
      const float sd_u = T > 1 ? sqrtf(v / (float)(T - 1)) : __builtin_nanf("");
      const float sharpe = (sd_u < 1e-8f) ? 0.f : mean / sd_u;
      if (pass == 0) {
        gp(J.scal)[SC_TRAIN_SHARPE] = sharpe;
      } else {
        gp(J.scal)[SC_SHARPE] = sharpe;
        gp(J.scal)[SC_MEAN] = mean;
        gp(J.scal)[SC_STD] = sqrtf(v / (float)T);
        float cum = 1.f, peak = 1.f, mdd = 0.f;
        for (int t = 0; t < T; ++t) {
          cum *= 1.f + ret[t];
          peak = t == 0 ? cum : fmaxf(peak, cum);
          mdd = fminf(mdd, (cum - peak) / peak);
        }
        gp(J.scal)[SC_MDD] = mdd;
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- launchers ------------
void launch_period_fwd(const LossJob* jobs, int njobs, int tmax, hipStream_t st) {
  hipLaunchKernelGGL(k_period_fwd, dim3(tmax, njobs), dim3(256), 0, st, jobs);
  HIP_OK(hipGetLastError());
}
void launch_asset(const LossJob* jobs, int njobs, int nmax, hipStream_t st) {
  hipLaunchKernelGGL(k_asset_part, dim3((nmax + 63) / 64, DLAP_TCH, njobs), dim3(256), 0, st, jobs);
  HIP_OK(hipGetLastError());
  hipLaunchKernelGGL(k_asset_red, dim3((nmax + 255) / 256, njobs), dim3(256), 0, st, jobs);
  HIP_OK(hipGetLastError());
}
void launch_period_bwd(const LossJob* jobs, int njobs, int tmax, hipStream_t st) {
  hipLaunchKernelGGL(k_period_bwd, dim3(tmax, njobs), dim3(256), 0, st, jobs);
  HIP_OK(hipGetLastError());
}
void launch_job_metrics(const LossJob* jobs, int njobs, hipStream_t st) {
  hipLaunchKernelGGL(k_job_metrics, dim3(njobs), dim3(256), 0, st, jobs);
  HIP_OK(hipGetLastError());
}
