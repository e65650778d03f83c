// Gradient finalisation, LSTM BPTT, clip + Adam, weight re-packing and device-side epoch
// bookkeeping (SURVEY §2.3 K7 backward, K8; §7.5 item 5 "host-sync-free orchestration").
//
// Reference semantics (`/root/reference/src/train.py:45-103,156-426`):
//   clip_grad_norm_(scope params, 1.0): coef = min(1, 1 / (||g||_2 + 1e-6)), g *= coef
//   torch.optim.Adam(lr, betas=(0.9, 0.999), eps=1e-8): m.lerp_(g, 0.1),
//     v = 0.999 v + 0.001 g^2, p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)
//   Two optimisers (sdf_net, moment_net) with independent step counts.
//   Best-model tracking with strict `epoch > ignore_epoch`, NaN never improves.
// Every reduction is a fixed-order sum (deterministic across runs).
#include "common.h"
#include "layout.h"
#include "update.h"
#include "loss.h"

// ============================================================ finalize ==================
// Sums the per-workgroup slabs of the MLP backward into the flat gradient vector and the
// per-row LSTM / moment-bias gradients into per-period sums. grid (nblocks, models).
__global__ __launch_bounds__(256) void k_finalize(const FinJob* __restrict__ jobs,
                                                  const ModelDesc* __restrict__ md, int phase,
                                                  int slab_stride) {
  const FinJob& J = jobs[blockIdx.y];
  const bool mom = phase == 2;
  const int ntile = mom ? md->ntile_m : md->ntile_s;
  const int nb_tiles = ntile * 16;
  const int nb_extra = (SLAB_EXTRA + 255) / 256;
  int b = blockIdx.x;
  if (b < nb_tiles) {
    const int ti = b >> 4, e = ((b & 15) << 8) + threadIdx.x;
    const GradTile& G = mom ? md->tile_m[ti] : md->tile_s[ti];
    const int o = e >> 6, i = (e & 63) + 64 * G.chunk;
    if (o >= G.out || i >= G.in) return;
    // position of this tile inside its slice's slab
    const int tps = 1;
    const int tpos = ti - G.slice * tps;
    const float* src = J.slab + (size_t)G.slice * J.nslab * slab_stride + tpos * 4096 + e;
    float s = 0.f;
#pragma unroll 16
    for (int k = 0; k < J.nslab; ++k) s += src[(size_t)k * slab_stride];
    J.grads[G.w_off + o * G.ld + G.col0 + i] = s;
    return;
  }
  b -= nb_tiles;
  if (b < nb_extra) {
    const int e = b * 256 + threadIdx.x;
    if (e >= SLAB_EXTRA) return;
    const int dst = mom ? md->extra_m[e] : md->extra_s[e];
    if (dst < 0) return;
    const float* src = J.slab + 1 * 4096 + e;   // slice-0 slabs (tps = 1)
    float s = 0.f;
#pragma unroll 16
    for (int k = 0; k < J.nslab; ++k) s += src[(size_t)k * slab_stride];
    J.grads[dst] = s;
    return;
  }
  b -= nb_extra;
  // per-period segment sums: one block per period, threads = (column d, row group)
  const int D = mom ? 64 : (md->nrnn > 0 ? md->Dm : 0);
  const int t = b;
  if (D == 0 || t >= J.T) return;
  __shared__ float red[256];
  int Dp = 1;
  while (Dp < D) Dp <<= 1;
  const int nrg = 256 / Dp, d = threadIdx.x % Dp, rg = threadIdx.x / Dp;
  const float* src = mom ? J.v : J.u;
  const int r0 = J.row_ptr[t], r1 = J.row_ptr[t + 1];
  float s = 0.f;
  if (d < D)
    for (int r = r0 + rg; r < r1; r += nrg) s += src[(size_t)r * D + d];
  red[threadIdx.x] = s;
  __syncthreads();
  if (rg == 0 && d < D) {
    float tot = 0.f;
    for (int g = 0; g < nrg; ++g) tot += red[g * Dp + d];
    if (mom) J.dab[t * 64 + d] = tot;
    else J.dpp[t * D + d] = tot;
  }
}

void launch_finalize(const FinJob* jobs, int njobs, const ModelDesc* md, const ModelDesc& mh,
                     int phase, int slab_stride, int tmax, hipStream_t st) {
  const bool mom = phase == 2;
  const int ntile = mom ? mh.ntile_m : mh.ntile_s;
  const int D = mom ? 64 : (mh.nrnn > 0 ? mh.Dm : 0);
  const int nb = ntile * 16 + (SLAB_EXTRA + 255) / 256 + (D > 0 ? tmax : 0);
  hipLaunchKernelGGL(k_finalize, dim3(nb, njobs), dim3(256), 0, st, jobs, md, phase, slab_stride);
  HIP_OK(hipGetLastError());
}

// ============================================================ packing ===================
DLAP_DEV int perm_u(int q, int j) { return j < 4 ? 4 * q + j : 16 + 4 * q + (j - 4); }

// Pack blob + aux of one model (all threads of the block participate).
DLAP_DEV void pack_model(const ModelDesc* __restrict__ md, const float* __restrict__ P,
                         bf16x8* blob, float* aux) {
  const MlpDims& D = md->md;
  const int KS1 = md->KS1, WMB = md->WMB, KSM = (WMB + 1) / 2;
  __bf16* out = reinterpret_cast<__bf16*>(blob);
  const int nel = D.blob_frags * 512;
  for (int e = threadIdx.x; e < nel; e += blockDim.x) {
    const int frag = e >> 9, lane = (e >> 3) & 63, j = e & 7;
    const int q = lane >> 4, n = lane & 15;
    float val = 0.f;
    if (frag < D.s_fwd) {                         // SDF layer 0, natural k
      const int u = frag / KS1, s = frag - u * KS1;
      const PackLayer& L = md->s[0];
      const int o = 16 * u + n, k = 32 * s + 8 * q + j;
      if (o < L.out && k < L.in) val = P[L.w_off + o * L.ld + k];
    } else if (frag < D.s_bwd) {                  // SDF chain forward
      const int loc = frag - D.s_fwd, jl = loc / 8 + 1, r = loc % 8, u = r >> 1, s = r & 1;
      const PackLayer& L = md->s[jl];
      const int o = 16 * u + n, i = 32 * s + perm_u(q, j);
      if (o < L.out && i < L.in) val = P[L.w_off + o * L.ld + i];
    } else if (frag < D.m_fwd0) {                 // SDF chain backward (W^T)
      const int loc = frag - D.s_bwd, jl = loc / 8 + 1, r = loc % 8, u = r >> 1, s = r & 1;
      const PackLayer& L = md->s[jl];
      const int i = 16 * u + n, o = 32 * s + perm_u(q, j);
      if (o < L.out && i < L.in) val = P[L.w_off + o * L.ld + i];
    } else if (frag < D.m_fwd) {                  // moment layer 0 (x columns only)
      const int loc = frag - D.m_fwd0, u = loc / KS1, s = loc - u * KS1;
      const PackLayer& L = md->m[0];
      const int o = 16 * u + n, k = 32 * s + 8 * q + j;
      if (o < L.out && k < L.in) val = P[L.w_off + o * L.ld + L.col0 + k];
    } else if (frag < D.m_bwd) {                  // moment chain forward
      const int per = WMB * KSM;
      const int loc = frag - D.m_fwd, jl = loc / per + 1, r = loc % per, u = r / KSM, s = r % KSM;
      const PackLayer& L = md->m[jl];
      const int o = 16 * u + n, i = 32 * s + perm_u(q, j);
      if (o < L.out && i < L.in) val = P[L.w_off + o * L.ld + i];
    } else {                                      // moment chain backward
      const int per = WMB * KSM;
      const int loc = frag - D.m_bwd, jl = loc / per + 1, r = loc % per, u = r / KSM, s = r % KSM;
      const PackLayer& L = md->m[jl];
      const int i = 16 * u + n, o = 32 * s + perm_u(q, j);
      if (o < L.out && i < L.in) val = P[L.w_off + o * L.ld + i];
    }
    out[e] = (__bf16)val;
  }
  for (int e = threadIdx.x; e < D.aux_floats; e += blockDim.x) {
    float val = 0.f;
    if (e < D.a_wo) {
      const int jl = e >> 6, o = e & 63;
      if (jl < md->nl_s && o < md->s[jl].out) val = P[md->s[jl].b_off + o];
    } else if (e < D.a_bo) {
      const int o = e - D.a_wo;
      if (o < md->s[md->nl_s - 1].out) val = P[md->so_w + o];
    } else if (e < D.a_pp) {
      if (e == D.a_bo) val = P[md->so_b];
    } else if (e < D.a_mb) {
      const int d = (e - D.a_pp) >> 6, o = (e - D.a_pp) & 63;
      const PackLayer& L = md->s[0];
      if (o < L.out && d < md->Dm) val = P[L.w_off + o * L.ld + md->F + d];
    } else {
      const int jl = (e - D.a_mb) >> 6, o = (e - D.a_mb) & 63;
      if (jl >= 1 && jl < md->nl_m && o < md->m[jl].out) val = P[md->m[jl].b_off + o];
    }
    aux[e] = val;
  }
}

__global__ __launch_bounds__(256) void k_pack(const UpdJob* __restrict__ jobs, const ModelDesc* __restrict__ md) {
  const UpdJob& J = jobs[blockIdx.x];
  pack_model(md, J.params, J.blob, J.aux);
}

void launch_pack(float* const*, const UpdJob* jobs, int njobs, const ModelDesc* md, hipStream_t st) {
  hipLaunchKernelGGL(k_pack, dim3(njobs), dim3(256), 0, st, jobs, md);
  HIP_OK(hipGetLastError());
}

// ============================================================ update ====================
__global__ __launch_bounds__(256) void k_update(const UpdJob* __restrict__ jobs,
                                                const ModelDesc* __restrict__ md, int phase, float lr,
                                                int apply) {
  const UpdJob& J = jobs[blockIdx.x];
  __shared__ float red[4];
  const bool mom = phase == 2;
  (void)apply;
  const int p0 = mom ? md->P_sdf : 0, p1 = mom ? md->P : md->P_sdf;
  float ss = 0.f;
  for (int i = p0 + threadIdx.x; i < p1; i += 256) { const float g = J.grads[i]; ss += g * g; }
  ss = block_sum<256>(ss, red);
  const float norm = sqrtf(ss);
  const float coef = fminf(1.f / (norm + 1e-6f), 1.f);
  const int step = J.adam_step[mom ? 1 : 0] + 1;
  const double bc1 = 1.0 - pow(0.9, (double)step);
  const double bc2 = 1.0 - pow(0.999, (double)step);
  const float step_size = (float)(lr / bc1);
  const float bc2s = (float)sqrt(bc2);
  for (int i = p0 + threadIdx.x; i < p1; i += 256) {
    const float g = J.grads[i] * coef;
    float m = J.m[i];
    m = m + 0.1f * (g - m);
    float v = 0.999f * J.v[i] + 0.001f * g * g;
    J.m[i] = m;
    J.v[i] = v;
    const float denom = sqrtf(v) / bc2s + 1e-8f;
    J.params[i] = J.params[i] - step_size * (m / denom);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    J.adam_step[mom ? 1 : 0] = step;
    J.gnorm[0] = norm;
  }
  __threadfence_block();
  __syncthreads();
  pack_model(md, J.params, J.blob, J.aux);
  __syncthreads();
  if (threadIdx.x == 0) J.drop_step[0] = J.drop_step[0] + 1;
}

void launch_update(const UpdJob* jobs, int njobs, const ModelDesc* md, int phase, float lr,
                   hipStream_t st, int apply) {
  hipLaunchKernelGGL(k_update, dim3(njobs), dim3(256), 0, st, jobs, md, phase, lr, apply);
  HIP_OK(hipGetLastError());
}

// ============================================================ epoch bookkeeping =========
__global__ __launch_bounds__(256) void k_epoch_end(const EpochJob* __restrict__ jobs, int phase,
                                                   int ignore_epoch, float sel, float res_factor, int P) {
  const EpochJob& J = jobs[blockIdx.x];
  __shared__ int dec[2];
  if (threadIdx.x == 0) {
    const int ep = J.ep[0], ep_ph = J.ep[1];
    float* row = J.hist + (size_t)ep * HIST_W;
    const float* tr = J.sc_train;
    const float lres = tr[SC_LRES] * res_factor;
    float tloss;
    if (phase == 1) tloss = tr[SC_LUNC] + lres;
    else if (phase == 2) tloss = -tr[SC_LCOND] + lres;
    else tloss = tr[SC_LCOND] + lres;
    for (int c = 0; c < HIST_W; ++c) row[c] = __builtin_nanf("");
    row[H_PHASE] = (float)phase;
    row[H_TRAIN_LOSS] = tloss;
    row[H_TRAIN_SHARPE] = tr[SC_TRAIN_SHARPE];
    row[H_TRAIN_LUNC] = phase == 2 ? 0.f : tr[SC_LUNC];
    row[H_TRAIN_LCOND] = phase == 1 ? 0.f : tr[SC_LCOND];
    row[H_TRAIN_LRES] = tr[SC_LRES];
    row[H_GNORM] = J.gnorm[0];
    int up_loss = 0, up_sr = 0;
    if (phase != 2) {
      const float* va = J.sc_valid;
      const float vloss = phase == 1 ? va[SC_LUNC] : va[SC_LCOND];
      row[H_VALID_LOSS] = vloss;
      row[H_VALID_SHARPE] = va[SC_SHARPE];
      row[H_VALID_LUNC] = va[SC_LUNC];
      row[H_VALID_LCOND] = va[SC_LCOND];
      row[H_VALID_MDD] = va[SC_MDD];
      row[H_VALID_MEAN] = va[SC_MEAN];
      row[H_VALID_STD] = va[SC_STD];
      if (J.sc_test) {
        const float* te = J.sc_test;
        row[H_TEST_LOSS] = phase == 1 ? te[SC_LUNC] : te[SC_LCOND];
        row[H_TEST_SHARPE] = te[SC_SHARPE];
        row[H_TEST_LUNC] = te[SC_LUNC];
        row[H_TEST_LCOND] = te[SC_LCOND];
        row[H_TEST_MDD] = te[SC_MDD];
        row[H_TEST_MEAN] = te[SC_MEAN];
        row[H_TEST_STD] = te[SC_STD];
      }
      if (ep_ph > ignore_epoch) {
        if (vloss < J.best[0]) { J.best[0] = vloss; up_loss = 1; }
        const float s = sel * va[SC_SHARPE];
        if (s > J.best[1]) { J.best[1] = s; up_sr = 1; }
      }
    } else {
      const float lc = tr[SC_LCOND];
      if (lc > J.best[2]) { J.best[2] = lc; up_loss = 1; }
    }
    row[H_BEST_LOSS] = (float)up_loss;
    row[H_BEST_SR] = (float)up_sr;
    if (up_loss) J.snap_flags[0] = 1;
    if (up_sr) J.snap_flags[1] = 1;
    J.ep[0] = ep + 1;
    J.ep[1] = ep_ph + 1;
    dec[0] = up_loss;
    dec[1] = up_sr;
  }
  __syncthreads();
  if (dec[0])
    for (int i = threadIdx.x; i < P; i += 256) J.snap_loss[i] = J.params[i];
  if (dec[1])
    for (int i = threadIdx.x; i < P; i += 256) J.snap_sharpe[i] = J.params[i];
}

void launch_epoch_end(const EpochJob* jobs, int njobs, int phase, int ignore_epoch, float sel,
                      float res_factor, int P, hipStream_t st) {
  hipLaunchKernelGGL(k_epoch_end, dim3(njobs), dim3(256), 0, st, jobs, phase, ignore_epoch, sel,
                     res_factor, P);
  HIP_OK(hipGetLastError());
}
