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
#include "finalize.h"

// ============================================================ finalize ==================
// The per-workgroup slab sums and per-period segment sums of the MLP backward (finalize.h),
// one block per element group / period. grid (nblocks, models).
__global__ __launch_bounds__(256) void k_finalize(const FinJob* __restrict__ jobs,
                                                  const ModelDesc* __restrict__ md, int phase,
                                                  int slab_stride, int b0) {
  // b0: first block of a partial launch (see launch_finalize)
  finalize_block(jobs[blockIdx.y], md, phase, slab_stride, blockIdx.x + b0);
}

void launch_finalize(const FinJob* jobs, int njobs, const ModelDesc* md, const ModelDesc& mh,
                     int phase, int slab_stride, int tmax, hipStream_t st, int part) {
  const bool mom = phase == 2;
  const int ntile = mom ? mh.ntile_m : mh.ntile_s;
  const int D = mom ? 64 : (mh.nrnn > 0 ? mh.Dm : 0);
  const int nslab = ntile * 64 + (SLAB_EXTRA + 63) / 64, nper = D > 0 ? tmax : 0;
  // part 0: everything; 1: the weight / bias slab sums; 2: the per-period segment sums (what
  // the LSTM backward reads), so part 1 can run beside the LSTM backward on another stream
  const int b0 = part == 2 ? nslab : 0;
  const int nb = part == 1 ? nslab : part == 2 ? nper : nslab + nper;
  if (nb == 0) return;
  hipLaunchKernelGGL(k_finalize, dim3(nb, njobs), dim3(256), 0, st, jobs, md, phase, slab_stride, b0);
  HIP_OK(hipGetLastError());
}

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

// Re-pack the bf16 MFMA weight fragments + fp32 aux of every model after an update.
// grid (ceil(elements / 256), models): one packed element per thread, gathered straight from
// the (L2-resident) parameter vector -- a single memory round trip per launch.
// Block 0 also advances the step counters (after every Adam block has read them).
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

// Index mode of the gathers: P[i] -> i + 1 (exact in fp32 below 2^24), padding stays 0.
struct PackIdx {
  DLAP_HD float operator[](int i) const { return (float)(i + 1); }
};

// src[e] = the parameter packed element e holds (-1: constant zero padding), evaluated on the
// host from the same gathers k_pack runs (once per engine; the engine inverts it into the
// scatter lists of k_adam).
void pack_index_host(const ModelDesc& mh, int* src) {
  const PackSpace S(&mh);
  for (int e = 0; e < S.total; ++e) src[e] = (int)pack_value(&mh, S, PackIdx{}, e) - 1;
}

__global__ __launch_bounds__(256) void k_pack(const UpdJob* __restrict__ jobs,
                                              const ModelDesc* __restrict__ md, int bump) {
  const UpdJob& J = jobs[blockIdx.y];
  const PackSpace S(md);
  const int e = blockIdx.x * 256 + threadIdx.x;
  const auto src = gp(static_cast<const float*>(J.params));
  const float dscale = J.dropout > 0.f ? 1.f / (1.f - J.dropout) : 1.f;
  if (e < S.total) pack_store(J, md, S, e, pack_value(md, S, src, e), dscale);
  // (a poisoned model's counters stay put, as in the fused k_adam, which returns early)
  if (bump && blockIdx.x == 0 && threadIdx.x == 0 && !prog_poisoned(J.prog)) {
    gp(J.adam_step)[bump - 1] = gp(J.adam_step)[bump - 1] + 1;
    gp(J.drop_step)[0] = gp(J.drop_step)[0] + 1;
  }
}

// One int written on the stream (module API: the dropout stream position of a model), so the
// host never touches device memory synchronously between calls. The store sits under a lane
// test (a vector store, not a scalar one).
__global__ __launch_bounds__(64) void k_set_int(int* p, int v) {
  if (threadIdx.x == 0) gp(p)[0] = v;
}

void launch_set_int(int* p, int v, hipStream_t st) {
  hipLaunchKernelGGL(k_set_int, dim3(1), dim3(64), 0, st, p, v);
  HIP_OK(hipGetLastError());
}

static int pack_blocks_of(const ModelDesc& mh) {
  return (pack_total(mh) + 255) / 256;
}

int pack_total(const ModelDesc& mh) {
  return mh.md.blob_frags * 512 + mh.md.aux_floats + (mh.proj_mp + 2) * mh.proj_np + mh.md.b0_frags * 512;
}


void launch_pack(float* const*, const UpdJob* jobs, int njobs, const ModelDesc* md, const ModelDesc& mh,
                 hipStream_t st) {
  hipLaunchKernelGGL(k_pack, dim3(pack_blocks_of(mh), njobs), dim3(256), 0, st, jobs, md, 0);
  HIP_OK(hipGetLastError());
}

// ============================================================ update ====================

// Clip-by-global-norm + Adam over the phase's scope. grid (blocks, models): every block
// reduces the full scope norm itself (fixed order -> identical in all blocks, no grid
// barrier) and updates its own ADAM_PB-parameter range.
#define ADAM_PB 1024
__global__ __launch_bounds__(256) void k_adam(const UpdJob* __restrict__ jobs,
                                              const ModelDesc* __restrict__ md, int phase, float lr) {
  const UpdJob& J = jobs[blockIdx.y];
  __shared__ float red[4];
  // a fused forward of this model gave up a wait (its outputs are incomplete): no update, now or
  // later (block-uniform; every launch that can bump the counters precedes this one on the stream)
  if (prog_poisoned(J.prog)) return;
  // the train split's scalars of this step, kept for the (possibly deferred) bookkeeping
  if (blockIdx.x == 0 && J.scal && threadIdx.x < SC_NSCAL) gp(J.scal_prev)[threadIdx.x] = gp(J.scal)[threadIdx.x];
  const bool mom = phase == 2;
  const int p0 = mom ? md->P_sdf : 0, p1 = mom ? md->P : md->P_sdf;
  const float* __restrict__ grads = gp(J.grads);
  // scope norm: the block's whole share of loads is issued before any use (register blocks of
  // ADAM_NB per thread), so the reduction costs ~one memory round trip per block of 256*ADAM_NB
  constexpr int ADAM_NB = 48;
  // bias corrections in double like torch's Python-float scalars, evaluated by every wave from
  // the (uniform) step count while the first norm loads are in flight
  const int step = gp(J.adam_step)[mom ? 1 : 0] + 1;
  const float lr_g = J.lr > 0.f ? J.lr : lr;
  float step_size = 0.f, bc2s = 1.f;
  float ss = 0.f;
  for (int b0 = p0; b0 < p1; b0 += 256 * ADAM_NB) {
    float gv[ADAM_NB];
#pragma unroll
    for (int k = 0; k < ADAM_NB; ++k) {
      const int i = b0 + k * 256 + threadIdx.x;
      gv[k] = grads[i < p1 ? i : p0];
    }
    if (b0 == p0) {
      const double bc1 = 1.0 - pow(0.9, (double)step);
      const double bc2 = 1.0 - pow(0.999, (double)step);
      step_size = (float)(lr_g / bc1);
      bc2s = (float)sqrt(bc2);
    }
#pragma unroll
    for (int k = 0; k < ADAM_NB; ++k) ss += (b0 + k * 256 + (int)threadIdx.x < p1) ? gv[k] * gv[k] : 0.f;
  }
  ss = block_sum<256>(ss, red);
  const float norm = sqrtf(ss);
  const float coef = fminf(1.f / (norm + 1e-6f), 1.f);
  const int i = p0 + blockIdx.x * ADAM_PB;
  float* __restrict__ pm = gp(J.m);
  float* __restrict__ pv = gp(J.v);
  float* __restrict__ pp = gp(J.params);
  // fused re-pack: every packed element holds exactly one parameter (pack_index_host), so the
  // thread that updates a parameter also writes its packed copies -- no second pass over the
  // parameter vector, no separate launch
  const bool fused = J.inv_code != nullptr;
  const PackSpace S(md);
  const float dscale = J.dropout > 0.f ? 1.f / (1.f - J.dropout) : 1.f;
  // every operand of the thread's ADAM_PB / 256 parameters (and their scatter lists) is requested
  // before the first use: one memory round trip
  constexpr int KPT = ADAM_PB / 256;
  float gq[KPT], mq[KPT], vq[KPT], pq[KPT];
  int cq[KPT][PACK_FAN];
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const int e = i + k * 256 + threadIdx.x, ec = e < p1 ? e : p0;
    gq[k] = grads[ec];
    mq[k] = pm[ec];
    vq[k] = pv[ec];
    pq[k] = pp[ec];
#pragma unroll
    for (int j = 0; j < PACK_FAN; ++j) cq[k][j] = fused ? gp(J.inv_code)[(size_t)ec * PACK_FAN + j] : -1;
  }
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
  if (blockIdx.x == 0 && threadIdx.x == 0) gp(J.gnorm)[0] = norm;
  // the last block to finish advances the step counters: every block has read them (above,
  // consumed before its increment), so no block of this launch can see the new values. Relaxed:
  // only that read must precede the increment (it has returned -- its value was used), and an
  // acquire / release at agent scope would write back and invalidate the XCD's L2.
  if (fused && threadIdx.x == 0) {
    const int done = __hip_atomic_fetch_add(J.upd_ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done == (int)gridDim.x - 1) {
      __hip_atomic_store(J.upd_ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      gp(J.adam_step)[mom ? 1 : 0] = gp(J.adam_step)[mom ? 1 : 0] + 1;
      gp(J.drop_step)[0] = gp(J.drop_step)[0] + 1;
    }
  }
}

void launch_update(const UpdJob* jobs, int njobs, const ModelDesc* md, const ModelDesc& mh, int phase,
                   float lr, hipStream_t st, bool fused) {
  const int n = phase == 2 ? mh.P - mh.P_sdf : mh.P_sdf;
  hipLaunchKernelGGL(k_adam, dim3((n + ADAM_PB - 1) / ADAM_PB, njobs), dim3(256), 0, st, jobs, md, phase,
                     lr);
  HIP_OK(hipGetLastError());
  if (fused) return;
  hipLaunchKernelGGL(k_pack, dim3(pack_blocks_of(mh), njobs), dim3(256), 0, st, jobs, md,
                     phase == 2 ? 2 : 1);
  HIP_OK(hipGetLastError());
}

// ============================================================ epoch bookkeeping =========
#define EPOCH_END_THREADS 1024
__global__ __launch_bounds__(EPOCH_END_THREADS) void k_epoch_end(const EpochJob* __restrict__ jobs, int phase,
                                                   int ignore_epoch, float sel, float res_factor, int P) {
  const EpochJob& J = jobs[blockIdx.x];
  __shared__ int dec[2];
  if (threadIdx.x == 0) {
    // every input is loaded before the first store: the stores below may alias them, so
    // loads left after a store would each pay a full memory round trip in sequence
    const bool hv = phase != 2 && J.sc_valid, ht = hv && J.sc_test;
    float tr[SC_NSCAL], va[SC_NSCAL], te[SC_NSCAL];
#pragma unroll
    for (int c = 0; c < SC_NSCAL; ++c) {
      tr[c] = gp(J.sc_train)[c];
      va[c] = hv ? gp(J.sc_valid)[c] : 0.f;
      te[c] = ht ? gp(J.sc_test)[c] : 0.f;
    }
    const int ep = gp(J.ep)[0], ep_ph = gp(J.ep)[1];
    const bool poisoned = prog_poisoned(J.prog);     // see k_adam: a NaN epoch, no bookkeeping
    const float gn = gp(J.gnorm)[0];
    const float best0 = gp(J.best)[0], best1 = gp(J.best)[1], best2 = gp(J.best)[2];
    // past the history capacity the row goes to a per-block scratch instead of out of bounds
    __shared__ float spill[HIST_W];
    float* row = ep < J.max_ep ? gp(J.hist) + (size_t)ep * HIST_W : spill;
    const float lres = tr[SC_LRES] * res_factor;
    float tloss;
    if (phase == 1) tloss = tr[SC_LUNC] + lres;
    else if (phase == 2) tloss = -tr[SC_LCOND] + lres;
    else tloss = tr[SC_LCOND] + lres;
    float r[HIST_W];
#pragma unroll
    for (int c = 0; c < HIST_W; ++c) r[c] = __builtin_nanf("");
    r[H_PHASE] = (float)phase;
    r[H_TRAIN_LOSS] = tloss;
    r[H_TRAIN_SHARPE] = tr[SC_TRAIN_SHARPE];
    r[H_TRAIN_LUNC] = phase == 2 ? 0.f : tr[SC_LUNC];
    r[H_TRAIN_LCOND] = phase == 1 ? 0.f : tr[SC_LCOND];
    r[H_TRAIN_LRES] = tr[SC_LRES];
    r[H_GNORM] = gn;
    int up_loss = 0, up_sr = 0;
    if (poisoned) {
#pragma unroll
      for (int c = 1; c < HIST_W; ++c) r[c] = __builtin_nanf("");
    } else if (hv) {
      const float vloss = phase == 1 ? va[SC_LUNC] : va[SC_LCOND];
      r[H_VALID_LOSS] = vloss;
      r[H_VALID_SHARPE] = va[SC_SHARPE];
      r[H_VALID_LUNC] = va[SC_LUNC];
      r[H_VALID_LCOND] = va[SC_LCOND];
      r[H_VALID_MDD] = va[SC_MDD];
      r[H_VALID_MEAN] = va[SC_MEAN];
      r[H_VALID_STD] = va[SC_STD];
      if (ht) {
        r[H_TEST_LOSS] = phase == 1 ? te[SC_LUNC] : te[SC_LCOND];
        r[H_TEST_SHARPE] = te[SC_SHARPE];
        r[H_TEST_LUNC] = te[SC_LUNC];
        r[H_TEST_LCOND] = te[SC_LCOND];
        r[H_TEST_MDD] = te[SC_MDD];
        r[H_TEST_MEAN] = te[SC_MEAN];
        r[H_TEST_STD] = te[SC_STD];
      }
      if (ep_ph > ignore_epoch) {
        if (vloss < best0) { gp(J.best)[0] = vloss; up_loss = 1; }
        const float s = sel * va[SC_SHARPE];
        if (s > best1) { gp(J.best)[1] = s; up_sr = 1; }
      }
    } else if (phase == 2) {
      const float lc = tr[SC_LCOND];
      if (lc > best2) { gp(J.best)[2] = lc; up_loss = 1; }
    }
    r[H_BEST_LOSS] = (float)up_loss;
    r[H_BEST_SR] = (float)up_sr;
#pragma unroll
    for (int c = 0; c < HIST_W; ++c) row[c] = r[c];
    if (up_loss) gp(J.snap_flags)[0] = 1;
    if (up_sr) gp(J.snap_flags)[1] = 1;
    gp(J.ep)[0] = ep + 1;
    gp(J.ep)[1] = ep_ph + 1;
    dec[0] = up_loss;
    dec[1] = up_sr;
  }
  __syncthreads();
  // snapshot copies: 16-byte accesses, every load of a thread issued before its stores (one
  // memory round trip for the whole vector instead of one per 256 floats)
  auto copy = [&](float* dst) {
    const auto src = gp(J.params);
    const auto d = gp(dst);
    const int P4 = ((reinterpret_cast<uintptr_t>(J.params) | reinterpret_cast<uintptr_t>(dst)) & 15) ? 0 : P >> 2;
    constexpr int U = 8;
    for (int i0 = threadIdx.x; i0 < P4; i0 += U * EPOCH_END_THREADS) {
      f32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * EPOCH_END_THREADS;
        v[u] = i < P4 ? ld4(src + 4 * i) : zero4();
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * EPOCH_END_THREADS;
        if (i < P4) *(DLAP_GLOBAL f32x4*)(d + 4 * i) = v[u];
      }
    }
    for (int i = 4 * P4 + threadIdx.x; i < P; i += EPOCH_END_THREADS) d[i] = src[i];
  };
  if (dec[0]) copy(J.snap_loss);
  if (dec[1]) copy(J.snap_sharpe);
}

// Phase start (reference: fresh best trackers per phase, `src/train.py:221-224`): best values
// (+inf loss, -inf Sharpe, -inf moment loss), snapshot flags and the in-phase epoch counter are
// reset on the stream, so a phase change needs no host synchronisation. One lane per model.
__global__ __launch_bounds__(64) void k_begin_phase(const EpochJob* __restrict__ jobs, int njobs) {
  const int g = blockIdx.x * 64 + threadIdx.x;
  if (g >= njobs) return;
  const EpochJob& J = jobs[g];
  gp(J.best)[0] = INFINITY;
  gp(J.best)[1] = -INFINITY;
  gp(J.best)[2] = -INFINITY;
  gp(J.snap_flags)[0] = 0;
  gp(J.snap_flags)[1] = 0;
  gp(J.ep)[1] = 0;
}

void launch_begin_phase(const EpochJob* jobs, int njobs, hipStream_t st) {
  hipLaunchKernelGGL(k_begin_phase, dim3((njobs + 63) / 64), dim3(64), 0, st, jobs, njobs);
  HIP_OK(hipGetLastError());
}

void launch_epoch_end(const EpochJob* jobs, int njobs, int phase, int ignore_epoch, float sel,
                      float res_factor, int P, hipStream_t st) {
  hipLaunchKernelGGL(k_epoch_end, dim3(njobs), dim3(EPOCH_END_THREADS), 0, st, jobs, phase, ignore_epoch, sel,
                     res_factor, P);
  HIP_OK(hipGetLastError());
}
