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
#include "pack_dev.h"

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

// Re-pack the bf16 MFMA weight fragments + fp32 aux of every model after an update.
// grid (ceil(elements / 256), models): one packed element per thread, gathered straight from
// the (L2-resident) parameter vector -- a single memory round trip per launch.
// Block 0 also advances the step counters (after every Adam block has read them).
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

// First launch of the split epoch graphs' evaluation graph (one wave): waits until the training
// graph's fused forward has counted `per` more finished evaluation recurrences (cnt[0], a
// running count) than this kernel has consumed (cnt[32]), then consumes them -- the
// evaluation towers behind it on this queue read those recurrences' outputs. Relaxed polls with
// s_sleep, bounded, one agent acquire. A wait that gives up poisons every model (its spin-timeout
// record, prog[48 g + 1]) and lets the graph run on: its results are then discarded (the host
// raises), and the counts stay in step (the bookkeeping still signals the training graph).
__global__ __launch_bounds__(64) void k_wait_count(int* cnt, int per, unsigned limit, int* prog, int nmodels) {
  const int seen = gp(cnt)[32];
  const unsigned want = (unsigned)(seen + per);
  unsigned spins = 0;
  bool ok = true;
  while ((unsigned)__builtin_amdgcn_readfirstlane(__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) - want >
         0x7fffffffu) {                                                // (wrap-safe "count < want")
    if (spins++ >= limit) { ok = false; break; }
    __builtin_amdgcn_s_sleep(2);
  }
  asm volatile("" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (threadIdx.x == 0) {
    gp(cnt)[32] = (int)want;
    if (!ok)
      for (int g = 0; g < nmodels; ++g) atomicAdd(prog + 48 * g + 1, 1);
  }
}

void launch_wait_count(int* cnt, int per, unsigned limit, int* prog, int nmodels, hipStream_t st) {
  hipLaunchKernelGGL(k_wait_count, dim3(1), dim3(64), 0, st, cnt, per, limit, prog, nmodels);
  HIP_OK(hipGetLastError());
}

// One wave; lane g (per 64 models) polls model g's update generation until it is one past what the
// evaluation graph consumed (wrap-safe), then ONE agent acquire and the consumed counts advance.
// Relaxed polls with s_sleep, bounded; a give-up poisons every model still waiting.
__global__ __launch_bounds__(64) void k_wait_gen(const UpdJob* __restrict__ jobs, int njobs, unsigned limit) {
  for (int g0 = 0; g0 < njobs; g0 += 64) {
    const int g = g0 + (int)threadIdx.x;
    const bool mine = g < njobs;
    int* ctr = mine ? jobs[g].tail_ctr : nullptr;
    const int want = mine ? gp(ctr)[TAIL_UPDSEEN] + 1 : 0;
    unsigned spins = 0;
    bool ok = true;
    while (true) {
      const bool done = !mine || __hip_atomic_load(ctr + TAIL_UPDGEN, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want >= 0;
      if (__all(done)) break;
      if (spins++ >= limit) { ok = done; break; }
      __builtin_amdgcn_s_sleep(2);
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (mine) {
      gp(ctr)[TAIL_UPDSEEN] = want;
      if (!ok) atomicAdd(const_cast<int*>(jobs[g].prog) + 1, 1);
    }
  }
}

__global__ __launch_bounds__(64) void k_gen_sync(const UpdJob* __restrict__ jobs, int njobs) {
  const int g = blockIdx.x * 64 + threadIdx.x;
  if (g >= njobs) return;
  int* ctr = jobs[g].tail_ctr;
  gp(ctr)[TAIL_UPDSEEN] = __hip_atomic_load(ctr + TAIL_UPDGEN, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - 1;
}

void launch_wait_gen(const UpdJob* jobs, int njobs, unsigned limit, hipStream_t st) {
  hipLaunchKernelGGL(k_wait_gen, dim3(1), dim3(64), 0, st, jobs, njobs, limit);
  HIP_OK(hipGetLastError());
}
void launch_gen_sync(const UpdJob* jobs, int njobs, hipStream_t st) {
  hipLaunchKernelGGL(k_gen_sync, dim3((njobs + 63) / 64), dim3(64), 0, st, jobs, njobs);
  HIP_OK(hipGetLastError());
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

// Clip-by-global-norm + Adam over the phase's scope (adam_block, pack_dev.h). grid (blocks,
// models): every block reduces the full scope norm itself (fixed order -> identical in all
// blocks, no grid barrier) and updates its own ADAM_PB-parameter range.
__global__ __launch_bounds__(256) void k_adam(const UpdJob* __restrict__ jobs,
                                              const ModelDesc* __restrict__ md, int phase, float lr) {
  const UpdJob& J = jobs[blockIdx.y];
  __shared__ float red[4];
  // a fused forward of this model gave up a wait (its outputs are incomplete): no update, now or
  // later (block-uniform; every launch that can bump the counters precedes this one on the stream)
  if (prog_poisoned(J.prog)) return;
  adam_block(J, md, phase, lr, blockIdx.x, gridDim.x, red, [] { return true; });
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
                                                   int ignore_epoch, float sel, float res_factor, int P,
                                                   int signal) {
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
  if (signal) {   // every read of params / write of this block done, then one count (agent release)
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_fetch_add(J.eval_gen, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
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
                      float res_factor, int P, hipStream_t st, int signal) {
  hipLaunchKernelGGL(k_epoch_end, dim3(njobs), dim3(EPOCH_END_THREADS), 0, st, jobs, phase, ignore_epoch, sel,
                     res_factor, P, signal);
  HIP_OK(hipGetLastError());
}
