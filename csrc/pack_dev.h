// Device helpers shared by k_update.hip (k_adam, k_pack) and the fused backward tail
// (k_rnn.hip, k_lstm_tail): the model's poison test, the packed-weight gathers / scatters and
// the clip + Adam block (adam_block).
#pragma once
#include "common.h"
#include "layout.h"
#include "update.h"
#include "loss.h"

DLAP_DEV bool prog_poisoned(const int* prog) {
  if (!prog) return false;
  const auto p = gp(prog);
  return (p[1] | p[16 + 1] | p[32 + 1]) != 0;
}

// ============================================================ packing ===================
DLAP_HD int perm_u(int q, int j) { return j < 4 ? 4 * q + j : 16 + 4 * q + (j - 4); }

// Pack one blob element / aux float of a model from its flat parameter vector.
template <typename PP>
DLAP_HD float pack_blob_elem(const ModelDesc* __restrict__ md, PP P, int e) {
  const MlpDims& D = md->md;
  const int KS1 = md->KSB, WMB = md->WMB, KSM = (WMB + 1) / 2;   // (no layer-0 range if KSB = 0)
  const int frag = e >> 9, lane = (e >> 3) & 63, j = e & 7;
  const int q = lane >> 4, n = lane & 15;
  float val = 0.f;
  if (frag < D.s_fwd) {                         // SDF layer 0, natural k = panel column
    const int u = frag / KS1, s = frag - u * KS1;
    const PackLayer& L = md->s[0];
    const int o = 16 * u + n, k = 32 * s + 8 * q + j;
    // panel columns [0, F): characteristics; [ppc, ppc + Dm): the per-period inputs
    const int c = k < md->F ? k : (k >= D.ppc && k < D.ppc + md->Dm ? md->F + (k - D.ppc) : -1);
    if (o < L.out && c >= 0) val = P[L.w_off + o * L.ld + c];
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
  } else if (frag < D.s_upp) {                  // moment chain backward
    const int per = WMB * KSM;
    const int loc = frag - D.m_bwd, jl = loc / per + 1, r = loc % per, u = r / KSM, s = r % KSM;
    const PackLayer& L = md->m[jl];
    const int i = 16 * u + n, o = 32 * s + perm_u(q, j);
    if (o < L.out && i < L.in) val = P[L.w_off + o * L.ld + i];
  } else if (frag < D.s_wo) {                   // SDF layer 0, per-period columns (W^T)
    const int loc = frag - D.s_upp, u = loc >> 1, s = loc & 1;
    const PackLayer& L = md->s[0];
    const int d = 16 * u + n, o = 32 * s + perm_u(q, j);
    if (o < L.out && d < md->Dm) val = P[L.w_off + o * L.ld + md->F + d];
  } else {                                      // SDF output row as row 0 of an A operand
    const int s = frag - D.s_wo, i = 32 * s + perm_u(q, j);
    if (n == 0 && i < md->s[md->nl_s - 1].out) val = P[md->so_w + i];
  }
  return val;
}
// whether blob fragment `frag` / aux float `e` belongs to a layer whose training copy carries
// the dropout scale (hidden layers >= 1 of both towers, forward and transposed, and wo)
DLAP_HD bool blob_scaled(const ModelDesc* __restrict__ md, int frag) {
  const MlpDims& D = md->md;
  return (frag >= D.s_fwd && frag < D.m_fwd0) || (frag >= D.m_fwd && frag < D.s_upp) ||
         (frag >= D.s_wo && frag < D.s_wo + 2);
}
DLAP_HD bool aux_scaled(const ModelDesc* __restrict__ md, int e) {
  return e >= md->md.a_wo && e < md->md.a_bo;
}

template <typename PP>
DLAP_HD float pack_aux_elem(const ModelDesc* __restrict__ md, PP P, int e) {
  const MlpDims& D = md->md;
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
  return val;
}

// Input-projection matrix for k_proj (ModelDesc::proj_mp): transposed, zero padded, biases in
// the last row, so k_proj can stage it with plain coalesced 16-byte loads.
template <typename PP>
DLAP_HD float pack_proj_elem(const ModelDesc* __restrict__ md, PP P, int f) {
  const int NP = md->proj_np, M = md->M;
  const int m = f / NP, o = f - m * NP;
  const int G4 = md->nrnn > 0 ? 4 * md->H : 0;
  const PackLayer& L0 = md->m[0];
  const int om = o - G4;
  if (m == md->proj_mp) {                       // bias rows: b_ih | b_m0, then b_hh | 0 (every
    if (o < G4) return P[md->lstm_b_ih[0] + o]; // packed element is one parameter, so the fused
    return om < md->cm1 ? P[L0.b_off + om] : 0.f;   // Adam can scatter each update itself)
  }
  if (m == md->proj_mp + 1) return o < G4 ? P[md->lstm_b_hh[0] + o] : 0.f;
  if (m >= M) return 0.f;
  if (o < G4) return P[md->lstm_w_ih[0] + o * M + m];
  return om < md->cm1 ? P[L0.w_off + om * L0.ld + m] : 0.f;
}

// Wide path: k_proj0's layer-0 weight fragments (natural k, as the tower blob's layer 0):
// fragment (u, s) with u < 4 the SDF W0[16u + n][32s + 8q + j], u >= 4 the moment layer 0's
// x columns; columns >= F and units beyond the layer width are zero.
template <typename PP>
DLAP_HD float pack_blob0_elem(const ModelDesc* __restrict__ md, PP P, int e) {
  const int KSX = md->md.KSX;
  const int frag = e >> 9, lane = (e >> 3) & 63, j = e & 7;
  const int q = lane >> 4, n = lane & 15;
  const int u = frag / KSX, s = frag - u * KSX;
  const int k = 32 * s + 8 * q + j;
  if (k >= md->F) return 0.f;
  if (u < 4) {
    const PackLayer& L = md->s[0];
    const int o = 16 * u + n;
    return o < L.out ? P[L.w_off + o * L.ld + k] : 0.f;
  }
  const PackLayer& L = md->m[0];
  const int o = 16 * (u - 4) + n;
  return o < L.out ? P[L.w_off + o * L.ld + L.col0 + k] : 0.f;
}

// The packed element space of a model, in order: blob (eval copy; the train copy sits nel
// further), aux (ditto), the input-projection matrix, the wide path's layer-0 fragments.
struct PackSpace {
  int nel, naux, nproj, total;
  DLAP_HD explicit PackSpace(const ModelDesc* __restrict__ md)
      : nel(md->md.blob_frags * 512), naux(nel + md->md.aux_floats),
        nproj(naux + (md->proj_mp + 2) * md->proj_np), total(nproj + md->md.b0_frags * 512) {}
};

// Value of packed element e gathered from the parameter vector (any P with operator[]).
template <typename PP>
DLAP_HD float pack_value(const ModelDesc* __restrict__ md, const PackSpace& S, PP P, int e) {
  if (e < S.nel) return pack_blob_elem(md, P, e);
  if (e < S.naux) return pack_aux_elem(md, P, e - S.nel);
  if (e < S.nproj) return pack_proj_elem(md, P, e - S.naux);
  return pack_blob0_elem(md, P, e - S.nproj);
}

// Store packed element e with value v: two copies of the blob / aux elements -- evaluation
// weights, then the training weights with the dropout scale 1/(1-p) folded into every layer fed
// by dropped-out activations (the towers then apply the bare keep mask; k_finalize scales those
// gradients back).
DLAP_DEV void pack_store(const UpdJob& J, const ModelDesc* __restrict__ md, const PackSpace& S, int e,
                         float v, float dscale) {
  if (e < S.nel) {
    const float vt = blob_scaled(md, e >> 9) ? v * dscale : v;
    if (md->md.fp32) {                                                // reference-precision towers
      ((DLAP_GLOBAL float*)(J.blob))[e] = v;
      ((DLAP_GLOBAL float*)(J.blob))[S.nel + e] = vt;
    } else {
      ((DLAP_GLOBAL __bf16*)(J.blob))[e] = (__bf16)v;
      ((DLAP_GLOBAL __bf16*)(J.blob))[S.nel + e] = (__bf16)vt;
    }
  } else if (e < S.naux) {
    const int a = e - S.nel;
    gp(J.aux)[a] = v;
    gp(J.aux)[md->md.aux_floats + a] = aux_scaled(md, a) ? v * dscale : v;
  } else if (e < S.nproj) {
    gp(J.wproj)[e - S.naux] = v;
  } else {
    if (md->md.fp32) ((DLAP_GLOBAL float*)(J.blob0))[e - S.nproj] = v;
    else ((DLAP_GLOBAL __bf16*)(J.blob0))[e - S.nproj] = (__bf16)v;
  }
}


// ============================================================ clip + Adam ===============
// One Adam block's share of the phase's update (k_adam, and the Adam blocks of the fused
// backward tail): the clip-by-global-norm scope norm -- reduced in full by every block in a
// fixed order, so it is the same value in all of them -- then parameters
// [p0 + bx ADAM_PB, + ADAM_PB) updated and written to their packed copies (the scatter lists:
// every packed element holds exactly one parameter, pack_index_host, so no second pass). The
// block's own operands (m, v, p, its scatter lists) are requested first; `wait()` runs before
// the first gradient load (k_adam: nothing; the tail: the wait for its last gradient writer and
// the evaluation branch) and returns false to skip the update (the model was poisoned). The
// last of the nblk blocks to finish advances the step counters: every block has read them
// (consumed before its increment), so none of this launch sees the new values -- relaxed, since
// only that read must precede the increment, and an agent acquire / release would write back
// and invalidate the XCD's L2. Returns true in thread 0 of that block.
// step_pre >= 0 (the fused tail): the step counters as read before this launch's first
// arrival (step_pre, drop_pre) -- block 0 advances them as soon as it is released (every block
// of the launch has read them by then), and no completion count is kept.
template <class W>
DLAP_DEV bool adam_block(const UpdJob& J, const ModelDesc* __restrict__ md, int phase, float lr, int bx,
                         int nblk, float* red, W&& wait, int step_pre = -1, int drop_pre = 0) {
  const bool mom = phase == 2;
  const int p0 = mom ? md->P_sdf : 0, p1 = mom ? md->P : md->P_sdf;
  const float* __restrict__ grads = gp(J.grads);
  float* __restrict__ pm = gp(J.m);
  float* __restrict__ pv = gp(J.v);
  float* __restrict__ pp = gp(J.params);
  const bool fused = J.inv_code != nullptr;
  const int i = p0 + bx * ADAM_PB;
  constexpr int KPT = ADAM_PB / 256;
  float gq[KPT], mq[KPT], vq[KPT], pq[KPT];
  int cq[KPT][PACK_FAN];
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const int e = i + k * 256 + threadIdx.x, ec = e < p1 ? e : p0;
    mq[k] = pm[ec];
    vq[k] = pv[ec];
    pq[k] = pp[ec];
#pragma unroll
    for (int j = 0; j < PACK_FAN; ++j) cq[k][j] = fused ? gp(J.inv_code)[(size_t)ec * PACK_FAN + j] : -1;
  }
  const bool go = wait();
  if (go) {
    // the train split's scalars of this step, kept for the (possibly deferred) bookkeeping
    if (bx == 0 && J.scal && threadIdx.x < SC_NSCAL) gp(J.scal_prev)[threadIdx.x] = gp(J.scal)[threadIdx.x];
    // scope norm: the block's whole share of loads is issued before any use (register blocks of
    // ADAM_NB per thread), so the reduction costs ~one memory round trip per 256 * ADAM_NB
    constexpr int ADAM_NB = 48;
    // bias corrections in double like torch's Python-float scalars, evaluated by every wave from
    // the (uniform) step count while the first norm loads are in flight
    const int step = (step_pre >= 0 ? step_pre : gp(J.adam_step)[mom ? 1 : 0]) + 1;
    if (step_pre >= 0 && bx == 0 && threadIdx.x == 0) {
      gp(J.adam_step)[mom ? 1 : 0] = step;
      gp(J.drop_step)[0] = drop_pre + 1;
    }
    const float lr_g = J.lr > 0.f ? J.lr : lr;
    float step_size = 0.f, bc2s = 1.f;
    float ss = 0.f;
    for (int b0 = p0; b0 < p1; b0 += 256 * ADAM_NB) {
      float gv[ADAM_NB];
#pragma unroll
      for (int k = 0; k < ADAM_NB; ++k) {
        const int e = b0 + k * 256 + threadIdx.x;
        gv[k] = grads[e < p1 ? e : p0];
      }
      if (b0 == p0) {
        const double bc1 = 1.0 - pow(0.9, (double)step);
        const double bc2 = 1.0 - pow(0.999, (double)step);
        step_size = (float)(lr_g / bc1);
        bc2s = (float)sqrt(bc2);
#pragma unroll
        for (int k = 0; k < KPT; ++k) {
          const int e = i + k * 256 + threadIdx.x;
          gq[k] = grads[e < p1 ? e : p0];
        }
      }
#pragma unroll
      for (int k = 0; k < ADAM_NB; ++k) ss += (b0 + k * 256 + (int)threadIdx.x < p1) ? gv[k] * gv[k] : 0.f;
    }
    ss = block_sum<256>(ss, red);
    const float norm = sqrtf(ss);
    const float coef = fminf(1.f / (norm + 1e-6f), 1.f);
    const PackSpace S(md);
    const float dscale = J.dropout > 0.f ? 1.f / (1.f - J.dropout) : 1.f;
#pragma unroll
    for (int k = 0; k < KPT; ++k) {
      const int e = i + k * 256 + threadIdx.x;
      if (e < p1) {
        const float g = gq[k] * coef;
        float m = mq[k];
        m = m + 0.1f * (g - m);
        const float v = 0.999f * vq[k] + 0.001f * g * g;
        pm[e] = m;
        pv[e] = v;
        const float denom = sqrtf(v) / bc2s + 1e-8f;
        const float pn = pq[k] - step_size * (m / denom);
        pp[e] = pn;
#pragma unroll
        for (int j = 0; j < PACK_FAN; ++j)
          if (cq[k][j] >= 0) pack_store(J, md, S, cq[k][j], pn, dscale);
      }
    }
    if (bx == 0 && threadIdx.x == 0) gp(J.gnorm)[0] = norm;
  }
  bool last = false;
  if (fused && step_pre < 0 && threadIdx.x == 0) {
    const int done = __hip_atomic_fetch_add(J.upd_ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done == nblk - 1) {
      __hip_atomic_store(J.upd_ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (go) {
        gp(J.adam_step)[mom ? 1 : 0] = gp(J.adam_step)[mom ? 1 : 0] + 1;
        gp(J.drop_step)[0] = gp(J.drop_step)[0] + 1;
      }
      last = true;
    }
  }
  return last;
}
